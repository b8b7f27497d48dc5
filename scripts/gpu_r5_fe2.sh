#!/bin/bash
# feature engineering profile (multiclass-text) after the native UTF-8 packing, then the MCT and headline benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/fe_profile.py multiclass-text 1000000 > gpurun_out/r5_fe2_mct.log 2>&1 || { tail -20 gpurun_out/r5_fe2_mct.log; exit 1; }
grep -a "FE train" gpurun_out/r5_fe2_mct.log
for cfg in multiclass-text binary-10m; do
  o=gpurun_out/r5_fe2_bench_${cfg}.log
  TMOG_FIT_PHASES=1 timeout -k 10 400 python3 -u bench.py --config $cfg --steps 5 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"holdout_error": [0-9.]*\|"step_s": [^]]*\|"FeatureEngineering": [0-9.]*'
done
