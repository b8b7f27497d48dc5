#!/bin/bash
# Round 6: feature-parallel resident loop, bf16 Gramian accuracy, mixed-storage LR and GPU CSV tests; headline with
# the lossless mixed LR pass vs plain fp32 (same box); 10M-row CSV ingest through the GPU parser.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6b
export TMPDIR=/tmp
O=gpurun_out/r6b
timeout -k 10 600 python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_dense_gemm_gpu.py tests/test_sanity_kernels_gpu.py tests/test_gpu_csv.py tests/test_linear_mixed_gpu.py \
  tests/test_learner_parallel.py tests/test_tree_resident_gpu.py tests/test_mlp.py tests/test_linear_bf16_gpu.py tests/test_sparse_linear_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for m in 1 0; do
  TMOG_LR_MIXED=$m timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 --verbose > $O/bench_mixed$m.log 2>&1 || { tail -20 $O/bench_mixed$m.log; exit 1; }
  echo "mixed=$m $(grep -a '^{' $O/bench_mixed$m.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"OpLogisticRegression": [0-9.]*\|"FeatureEngineering": [0-9.]*\|"ModelRefit": [0-9.]*' | tr '\n' ' ')"
done
TMOG_INGEST_PROFILE=1 timeout -k 10 600 python3 -u bench.py --ingest csv --steps 2 --warmup 1 --verbose > $O/ingest_csv.log 2>&1 || { tail -20 $O/ingest_csv.log; exit 1; }
grep -a "gpu-csv\|ingest-profile\|\[ingest\]" $O/ingest_csv.log | tail -4
echo "csv $(grep -a '^{' $O/ingest_csv.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*' | tr '\n' ' ')"
