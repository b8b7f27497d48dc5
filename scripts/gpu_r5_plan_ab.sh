#!/bin/bash
# Headline A/B on one box: level-planner scratch in LDS (default) vs global memory, and 5 / 6 boosting parts.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --verbose > gpurun_out/r5p_$tag.log 2>&1 || { tail -20 gpurun_out/r5p_$tag.log; return 1; }
  echo "$tag $(grep -a '^{' gpurun_out/r5p_$tag.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*\|"OpLogisticRegression": [0-9.]*\|"OpRandomForestClassifier": [0-9.]*' | tr '\n' ' ')"
}
run base || exit 1
run nolds TMOG_PLAN_LDS=0 || exit 1
run pipe6 TMOG_XGB_PIPE=6 || exit 1
run nolds2 TMOG_PLAN_LDS=0 || exit 1
run base2 || exit 1
