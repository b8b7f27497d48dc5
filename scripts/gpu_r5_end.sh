#!/bin/bash
# end-of-session check: GPU suite + smoke, packing microbench, FE profile, multiclass-text / lr-rf-1m / headline benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_end_suite.log 2>&1 || { tail -40 gpurun_out/r5_end_suite.log; exit 1; }
tail -1 gpurun_out/r5_end_suite.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_end_smoke.log 2>&1 || { tail -20 gpurun_out/r5_end_smoke.log; exit 1; }
tail -1 gpurun_out/r5_end_smoke.log
timeout -k 10 300 python3 -u scripts/bench_pack.py > gpurun_out/r5_end_pack.log 2>&1 || { tail -20 gpurun_out/r5_end_pack.log; exit 1; }
cat gpurun_out/r5_end_pack.log | grep -v amdgpu.ids
timeout -k 10 300 python3 -u scripts/fe_profile.py multiclass-text 1000000 > gpurun_out/r5_end_fe_mct.log 2>&1 || { tail -20 gpurun_out/r5_end_fe_mct.log; exit 1; }
grep -a "FE train" gpurun_out/r5_end_fe_mct.log | cut -c1-200
for cfg in multiclass-text lr-rf-1m binary-10m; do
  o=gpurun_out/r5_end_bench_${cfg}.log
  timeout -k 10 400 python3 -u bench.py --config $cfg --steps 5 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  echo "$cfg $(grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"holdout_error": [0-9.]*\|"FeatureEngineering": [0-9.]*' | tr '\n' ' ')"
done
