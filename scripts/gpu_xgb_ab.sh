#!/bin/bash
# In-process A/B of the XGBoost phase: $AB_A vs $AB_B (env assignments), $AB_REPS alternations.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${AB_T:-600} python -u scripts/debug/xgb_ab.py "$AB_A" "$AB_B" ${AB_REPS:-3} > gpurun_out/xgb_ab.log 2>&1; rc=$?
cat gpurun_out/xgb_ab.log | tail -n 12
exit $rc
