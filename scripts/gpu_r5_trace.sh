#!/bin/bash
# Round 5: kernel traces of the headline and of the XGBoost-only selector (warm-up + 1 step each), with the
# per-part XGBoost host profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TMOG_XGB_PROFILE=1 timeout -k 10 200 python3 -u bench.py --models OpXGBoostClassifier --steps 2 --warmup 1 --verbose \
  > gpurun_out/r5_xgb_only.log 2>&1 || { tail -20 gpurun_out/r5_xgb_only.log; exit 1; }
grep -a '^{' gpurun_out/r5_xgb_only.log | grep -o '"value": [0-9.]*\|"step_s": [^]]*'
grep -a 'xgb-profile' gpurun_out/r5_xgb_only.log | tail -2
bash scripts/gpu_r4_trace.sh r5xgb "--models OpXGBoostClassifier" || exit $?
bash scripts/gpu_r4_trace.sh r5full ""
