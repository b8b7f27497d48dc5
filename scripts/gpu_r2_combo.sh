#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_sanity_kernels_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/c_test.log 2>&1 || { tail -30 gpurun_out/c_test.log; exit 1; }
tail -3 gpurun_out/c_test.log
bash scripts/gpu_pmc_bench.sh > gpurun_out/c_pmc.log 2>&1
