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
