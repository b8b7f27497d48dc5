#!/bin/bash
# New tree tests (long CSR lists, wide) + host cProfile of a warmed headline step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/t2_test.log 2>&1 || { tail -30 gpurun_out/t2_test.log; exit 1; }
tail -3 gpurun_out/t2_test.log
PROF_ROWS=10000000 BENCH_ARGS="--warmup 1" PROF_T=400 bash scripts/gpu_pyprof.sh
