#!/bin/bash
# Lanes / side-stream A/B on the headline (same box): each argument "LANES:SIDE".
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; STEPS=$2; shift 2
mkdir -p gpurun_out
for C in "$@"; do
  L=${C%%:*}; S=${C##*:}
  TMOG_LEARNER_LANES=$L TMOG_SIDE_STREAMS=$S TMOG_WATCHDOG_S=10 timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 1 --verbose > gpurun_out/lanes_${TAG}_${L}_${S}.log 2>&1 || { echo "$C failed"; tail -20 gpurun_out/lanes_${TAG}_${L}_${S}.log; exit 1; }
  echo "[lanes=$L side=$S] $(grep -a '^{' gpurun_out/lanes_${TAG}_${L}_${S}.log | grep -o '"value": [0-9.]*\|"step_s": \[[^]]*\]\|"stalls": \[' | tr '\n' ' ')"
done
