#!/bin/bash
# The whole GPU test suite in one pytest process (per-test timeout), then smoke().
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread tests/ > gpurun_out/all_${TAG}.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/all_${TAG}.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
src=$?
tail -3 gpurun_out/smoke_${TAG}.log
exit $(( rc > src ? rc : src ))
