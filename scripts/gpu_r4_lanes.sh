#!/bin/bash
# Learner lanes A/B on the headline (same box): off, 2, 3 lanes; per-step times and watchdog stalls in each line.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; STEPS=${2:-3}
mkdir -p gpurun_out
for L in 1 2 3; do
  TMOG_LEARNER_LANES=$L TMOG_WATCHDOG_S=10 timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 1 --verbose > gpurun_out/lanes_${TAG}_$L.log 2>&1 || { echo "lanes=$L failed"; tail -20 gpurun_out/lanes_${TAG}_$L.log; exit 1; }
  echo "[lanes=$L] $(grep -a '^{' gpurun_out/lanes_${TAG}_$L.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"step_s": \[[^]]*\]\|"stalls": \[' | tr '\n' ' ')"
done
