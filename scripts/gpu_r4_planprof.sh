#!/bin/bash
# Phase timing of the device level planner (TMOG_PLAN_PROFILE) on the XGBoost-only selector.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
mkdir -p gpurun_out
TMOG_PLAN_PROFILE=1 TMOG_XGB_PROFILE=1 timeout -k 10 300 python -u bench.py --models OpXGBoostClassifier --steps 1 --warmup 1 --verbose > gpurun_out/pp_${TAG}.log 2>&1
rc=$?
grep -a "xgb-profile" gpurun_out/pp_${TAG}.log | tail -n 2
grep -a '^{' gpurun_out/pp_${TAG}.log | tail -c 600
exit $rc
