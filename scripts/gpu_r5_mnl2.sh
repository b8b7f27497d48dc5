#!/bin/bash
# wide OWL-QN direction kernel (multinomial columns) + multiclass-text bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_linear_kernels.py tests/test_linear_bf16_gpu.py -m gpu > gpurun_out/r5_mnl2_tests.log 2>&1 || { tail -40 gpurun_out/r5_mnl2_tests.log; exit 1; }
tail -1 gpurun_out/r5_mnl2_tests.log
o=gpurun_out/r5_mnl2_bench_mct.log
TMOG_FIT_PHASES=1 timeout -k 10 400 python3 -u bench.py --config multiclass-text --steps 5 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_error": [0-9.]*\|"step_s": [^]]*\|"timings": {[^}]*}'
