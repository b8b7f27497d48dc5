#!/bin/bash
# 3 boosting parts (2 jobs each) vs 4 parts merged into the 3 streams left beside the other lane (3 + 2 + 1 jobs)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --verbose > gpurun_out/r5p3_$tag.log 2>&1 || { tail -20 gpurun_out/r5p3_$tag.log; return 1; }
  echo "$tag $(grep -a '^{' gpurun_out/r5p3_$tag.log | grep -o '"value": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*\|"holdout_aupr": [0-9.]*' | tr '\n' ' ')"
}
for i in 1 2 3; do
  run p3_$i TMOG_XGB_PIPE=3 || exit 1
  run base_$i || exit 1
done
