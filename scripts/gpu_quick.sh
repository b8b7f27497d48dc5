#!/bin/bash
# GPU tests + tree microbenchmark.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/bench_trees.py > gpurun_out/trees_gh.log 2>&1 || { tail -20 gpurun_out/trees_gh.log; exit 1; }
tail -1 gpurun_out/trees_gh.log
timeout -k 10 300 python benchmarks/bench_trees.py --rf --trees 50 --depth 12 > gpurun_out/trees_rf.log 2>&1 || { tail -20 gpurun_out/trees_rf.log; exit 1; }
tail -1 gpurun_out/trees_rf.log
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py --rows ${ROWS:-10000000} --warmup 0 --steps 1 --verbose > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log
fi
