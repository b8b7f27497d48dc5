#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_metric_kernels_gpu.py > gpurun_out/r5f_tests.log 2>&1 || { tail -30 gpurun_out/r5f_tests.log; exit 1; }
tail -1 gpurun_out/r5f_tests.log
timeout -k 10 200 python -u scripts/bench_metric.py > gpurun_out/r5f_bench_metric.log 2>&1 || { tail -20 gpurun_out/r5f_bench_metric.log; exit 1; }
cat gpurun_out/r5f_bench_metric.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --verbose > gpurun_out/r5f_full.log 2>&1 || { tail -20 gpurun_out/r5f_full.log; exit 1; }
grep -a '^{' gpurun_out/r5f_full.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"best_model": "[A-Za-z]*"\|"timings": {[^}]*}'
