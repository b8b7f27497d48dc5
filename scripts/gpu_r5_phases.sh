#!/bin/bash
# Phase breakdown of the XGBoost learner: setup / boosting loop (per part host profile) / validation predict.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TMOG_FIT_PHASES=1 TMOG_XGB_PROFILE=1 timeout -k 10 200 python3 -u bench.py --models OpXGBoostClassifier --steps 1 --warmup 1 --verbose \
  > gpurun_out/r5p_xgb.log 2>&1 || { tail -20 gpurun_out/r5p_xgb.log; exit 1; }
grep -a 'xgb-profile' gpurun_out/r5p_xgb.log
grep -a '^{' gpurun_out/r5p_xgb.log | grep -o '"value": [0-9.]*\|"fit_phases": {[^}]*}\|"timings": {[^}]*}'
TMOG_FIT_PHASES=1 timeout -k 10 200 python3 -u bench.py --steps 1 --warmup 1 --verbose \
  > gpurun_out/r5p_full.log 2>&1 || { tail -20 gpurun_out/r5p_full.log; exit 1; }
grep -a '^{' gpurun_out/r5p_full.log | grep -o '"value": [0-9.]*\|"fit_phases": {[^}]*}\|"timings": {[^}]*}'
