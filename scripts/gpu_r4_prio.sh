#!/bin/bash
# Lane-priority A/B on the headline (same box): the lane / stream tests, then TMOG_LANE_PRIO=0 / 1 / 0 / 1.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; STEPS=${2:-5}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_concurrent_lanes.py tests/test_watchdog_streams.py > gpurun_out/prio_${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/prio_${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/prio_${TAG}_tests.log
for P in 0 1 0 1; do
  TMOG_LANE_PRIO=$P TMOG_WATCHDOG_S=10 timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 1 --verbose > gpurun_out/prio_${TAG}_${P}.log 2>&1 || { echo "prio $P failed"; tail -20 gpurun_out/prio_${TAG}_${P}.log; exit 1; }
  echo "[prio=$P] $(grep -a '^{' gpurun_out/prio_${TAG}_${P}.log | grep -o '"value": [0-9.]*\|"step_s": \[[^]]*\]\|"timings": {[^}]*}' | tr '\n' ' ')"
done
