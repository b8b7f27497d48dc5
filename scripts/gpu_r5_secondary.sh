#!/bin/bash
# the secondary BASELINE configs with the round-5 defaults (bf16 linear learners)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in lr-rf-1m regression-100m; do
  o=gpurun_out/r5_final_${cfg}.log
  TMOG_FIT_PHASES=1 timeout -k 10 600 python3 -u bench.py --config $cfg --steps 3 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_[a-z]*": [0-9.]*\|"step_s": [^]]*\|"best_model": "[A-Za-z]*"'
done
