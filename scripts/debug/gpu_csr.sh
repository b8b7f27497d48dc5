#!/bin/bash
# GPU check of the CSR histogram path: engine + kernel tests, then the 10M bench with / without it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/csr_tests.log 2>&1; rc=$?
tail -5 gpurun_out/csr_tests.log
[ $rc -eq 0 ] || exit $rc
AB_ENV=TMOG_TREE_CSR=0 bash scripts/debug/bench_ab.sh
