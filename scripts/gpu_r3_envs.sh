#!/bin/bash
# Headline bench under several env settings on one box (A/B/C...): bash scripts/gpu_r3_envs.sh TAG "A=1" "A=0 B=2" ...
# Optional GPU tests first (PYTEST_K selects). Every step has its own time limit; the first failure ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
STEPS=${STEPS:-5}
mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" > gpurun_out/${TAG}_gputest.log 2>&1 || exit $?
  tail -n 2 gpurun_out/${TAG}_gputest.log
fi
i=0
for e in "$@"; do
  env $e timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 2 --verbose ${BENCH_ARGS} > gpurun_out/${TAG}_$i.log 2>&1 || exit $?
  echo "[$i] $e"; tail -c 400 gpurun_out/${TAG}_$i.log; echo
  i=$((i+1))
done
