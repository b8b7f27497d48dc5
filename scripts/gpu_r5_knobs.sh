#!/bin/bash
# Headline A/B of scheduling knobs on one box: early-stopping lag, lane priority, boosting parts.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --verbose > gpurun_out/r5k_$tag.log 2>&1 || { tail -20 gpurun_out/r5k_$tag.log; return 1; }
  echo "$tag $(grep -a '^{' gpurun_out/r5k_$tag.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*\|"OpLogisticRegression": [0-9.]*\|"OpRandomForestClassifier": [0-9.]*' | tr '\n' ' ')"
}
run base || exit 1
run lag4 TMOG_ES_LAG=4 || exit 1
run lag8 TMOG_ES_LAG=8 || exit 1
run prio TMOG_LANE_PRIO=1 || exit 1
run pipe3 TMOG_XGB_PIPE=3 || exit 1
run base2 || exit 1
