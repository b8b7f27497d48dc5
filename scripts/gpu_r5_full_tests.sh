#!/bin/bash
# the whole GPU test suite, one process, then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_gpu_suite.log 2>&1 || { tail -40 gpurun_out/r5_gpu_suite.log; exit 1; }
tail -3 gpurun_out/r5_gpu_suite.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke.log 2>&1 || { tail -20 gpurun_out/r5_smoke.log; exit 1; }
tail -1 gpurun_out/r5_smoke.log
