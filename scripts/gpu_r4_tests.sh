#!/bin/bash
# Selected GPU tests (one pytest process, per-test timeout): bash scripts/gpu_r4_tests.sh TAG "<test paths / -k>"
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread "$@" > gpurun_out/t_${TAG}.log 2>&1
rc=$?
tail -n 30 gpurun_out/t_${TAG}.log
exit $rc
