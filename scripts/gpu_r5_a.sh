#!/bin/bash
# Round 5, first call: allocation-failure / NaN-ingest / resident-tree GPU tests, then the regression-100m
# config with a 20M-row training sample under default lanes (the round-4 fault), then the headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread \
  tests/test_native_alloc_gpu.py tests/test_tree_resident_gpu.py tests/test_columnar_ingest.py \
  > gpurun_out/r5a_tests.log 2>&1 || { tail -40 gpurun_out/r5a_tests.log; exit 1; }
tail -n 5 gpurun_out/r5a_tests.log
timeout -k 10 600 python -u bench.py --config regression-100m --max-training-sample 20000000 --steps 1 --warmup 1 \
  --verbose > gpurun_out/r5a_reg20m.log 2>&1
rc=$?
grep -a '^{' gpurun_out/r5a_reg20m.log | grep -o '"value": [0-9.]*\|"holdout_[a-z]*": [0-9.e-]*\|"configs_evaluated": [0-9]*\|"peak_hbm_gb_per_gpu": [0-9.]*'
[ $rc -ne 0 ] && { tail -30 gpurun_out/r5a_reg20m.log; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --verbose > gpurun_out/r5a_bench.log 2>&1 || { tail -30 gpurun_out/r5a_bench.log; exit 1; }
grep -a '^{' gpurun_out/r5a_bench.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"timings": {[^}]*}\|"step_s": [^]]*'
