#!/bin/bash
# A/B of the line-search acceptance check every 1 / 2 / 3 trials (TMOG_LS_BATCH) on lr-rf-1m and the MCT config
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 1 2 3 1 2 3; do
  o=gpurun_out/r5_ls_ab_$b.log
  TMOG_LS_BATCH=$b timeout -k 10 300 python3 -u bench.py --config lr-rf-1m --steps 5 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  echo "lrrf batch=$b $(grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"OpLogisticRegression": [0-9.]*' | tr '\n' ' ')"
done
for b in 1 2; do
  o=gpurun_out/r5_ls_ab_mct_$b.log
  TMOG_LS_BATCH=$b timeout -k 10 300 python3 -u bench.py --config multiclass-text --steps 3 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  echo "mct batch=$b $(grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_error": [0-9.]*\|"OpLogisticRegression": [0-9.]*' | tr '\n' ' ')"
done
