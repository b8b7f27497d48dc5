#!/bin/bash
# XGBoost-only selector A/B over environment settings: bash scripts/gpu_r4_xgb_ab.sh TAG STEPS "ENV1" "ENV2" ...
# (each ENV is a space-separated list of VAR=value, "-" for none); one bench per setting, in order.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; STEPS=$2; shift 2
mkdir -p gpurun_out
k=0
for E in "$@"; do
  k=$((k+1))
  [ "$E" = "-" ] && E=""
  env $E timeout -k 10 300 python -u bench.py --models OpXGBoostClassifier --steps $STEPS --warmup 1 --verbose > gpurun_out/ab_${TAG}_$k.log 2>&1 || { echo "setting $k ($E) failed"; tail -5 gpurun_out/ab_${TAG}_$k.log; exit 1; }
  echo "[$k] $E :: $(grep -a '^{' gpurun_out/ab_${TAG}_$k.log | grep -o '"value": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*\|"holdout_aupr": [0-9.]*' | tr '\n' ' ')"
done
