#!/bin/bash
# Selected GPU tests, then (unless they crashed / timed out) a short headline bench:
#   bash scripts/gpu_r4_combo.sh TAG STEPS "<pytest args>"
# Test failures (exit 1) still run the bench; a crash, abort or time limit ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; STEPS=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread "$@" > gpurun_out/t_${TAG}.log 2>&1
rc=$?
tail -n 25 gpurun_out/t_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 2 --verbose > gpurun_out/b_${TAG}.log 2>&1
brc=$?
tail -c 3000 gpurun_out/b_${TAG}.log
exit $(( rc > brc ? rc : brc ))
