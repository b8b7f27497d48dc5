#!/bin/bash
# Round 6: the FeatureEngineering swing cases of VERDICT r5 #4 (XGBoost-only selector at 10M rows) and the
# regression-100m config with a 20M training sample (budgeted tree batches: no OOM, peak HBM reported).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 200 python3 -u scripts/bench_dense.py > $O/bench_dense.log 2>&1 || { tail -20 $O/bench_dense.log; exit 1; }
cat $O/bench_dense.log
timeout -k 10 400 python3 -u bench.py --models OpXGBoostClassifier --steps 2 --warmup 1 --verbose > $O/xgb_alone.log 2>&1 || { tail -20 $O/xgb_alone.log; exit 1; }
echo "xgb-alone $(grep -a '^{' $O/xgb_alone.log | grep -o '"value": [0-9.]*\|"FeatureEngineering": [0-9.]*\|"ModelRefit": [0-9.]*' | tr '\n' ' ')"
timeout -k 10 900 python3 -u bench.py --config regression-100m --max-training-sample 20000000 --steps 1 --warmup 1 --verbose > $O/reg100m_20m.log 2>&1 || { tail -30 $O/reg100m_20m.log; exit 1; }
echo "reg100m-20m $(grep -a '^{' $O/reg100m_20m.log | grep -o '"value": [0-9.]*\|"peak_hbm_gb_per_gpu": [0-9.]*' | tr '\n' ' ')"
grep -a -i "oom\|out of memory" $O/reg100m_20m.log | head -3 || true
for m in 1 0; do
  TMOG_DENSE_MFMA=$m timeout -k 10 400 python3 -u bench.py --config multiclass-text --steps 3 --warmup 1 --verbose > $O/mct_dense$m.log 2>&1 || { tail -20 $O/mct_dense$m.log; exit 1; }
  echo "mct dense=$m $(grep -a '^{' $O/mct_dense$m.log | grep -o '"value": [0-9.]*\|"holdout_error": [0-9.]*\|"OpLogisticRegression": [0-9.]*' | tr '\n' ' ')"
done
# projection FE outlier check: the rank-0 share of world 2 and 4 over 3 timed steps (r6c showed a 1.4 s pivot
# transform / 2.2 s selector fit in single-step runs)
timeout -k 10 400 python3 -u scripts/project_schedule.py --world 2 --ranks 0 --steps 3 --out $O/proj2s3 > $O/proj2s3.out 2>&1 || { tail -20 $O/proj2s3.out; exit 1; }
tail -1 $O/proj2s3.out
grep -a -o '"step_s": \[[^]]*\]' $O/proj2s3/rank0.log
timeout -k 10 400 python3 -u scripts/project_schedule.py --world 4 --ranks 0 --steps 3 --out $O/proj4s3 > $O/proj4s3.out 2>&1 || { tail -20 $O/proj4s3.out; exit 1; }
tail -1 $O/proj4s3.out
grep -a -o '"step_s": \[[^]]*\]' $O/proj4s3/rank0.log
