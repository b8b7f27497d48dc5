#!/bin/bash
# Compact histogram matrix (TMOG_HIST_COMPACT): tree GPU tests, then XGBoost-only and headline A/B on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread \
  tests/test_tree_resident_gpu.py tests/test_native_alloc_gpu.py tests/test_tree_wide_rows.py tests/test_tree_engine.py tests/test_tree_capacity.py \
  > gpurun_out/r5c_tests.log 2>&1 || { tail -40 gpurun_out/r5c_tests.log; exit 1; }
tail -n 3 gpurun_out/r5c_tests.log
for v in 1 0 1 0; do
  TMOG_HIST_COMPACT=$v timeout -k 10 200 python3 -u bench.py --models OpXGBoostClassifier --steps 3 --warmup 1 --verbose \
    > gpurun_out/r5c_xgb_$v.log 2>&1 || { tail -20 gpurun_out/r5c_xgb_$v.log; exit 1; }
  echo "compact=$v $(grep -a '^{' gpurun_out/r5c_xgb_$v.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*' | tr '\n' ' ')"
done
for v in 1 0; do
  TMOG_HIST_COMPACT=$v timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --verbose > gpurun_out/r5c_full_$v.log 2>&1 || exit 1
  echo "full compact=$v $(grep -a '^{' gpurun_out/r5c_full_$v.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*' | tr '\n' ' ')"
done
