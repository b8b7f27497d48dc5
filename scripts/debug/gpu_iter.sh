#!/bin/bash
# GPU iteration: tree tests, kernel-stats profile of the 10M bench, then an A/B of $AB_ENV.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1; rc=$?
tail -3 gpurun_out/iter_tests.log
[ $rc -eq 0 ] || exit $rc
PROF_ROWS=10000000 bash scripts/gpu_prof.sh > /dev/null || exit $?
AB_ENV="$AB_ENV" bash scripts/debug/bench_ab.sh
