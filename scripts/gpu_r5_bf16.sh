#!/bin/bash
# bf16 linear objective: numerics tests, then the headline and lr-rf-1m at fp32 and at bf16 (same box), with
# per-phase fit times.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_linear_bf16_gpu.py tests/test_sanity_kernels_gpu.py > gpurun_out/r5_bf16_tests.log 2>&1 || { tail -40 gpurun_out/r5_bf16_tests.log; exit 1; }
tail -1 gpurun_out/r5_bf16_tests.log
for cfg in ${CFGS:-binary-10m lr-rf-1m}; do
for dt in fp32 bf16; do
  o=gpurun_out/r5_bench_${cfg}_$dt.log
  TMOG_FIT_PHASES=1 timeout -k 10 400 python3 -u bench.py --config $cfg --dtype $dt --steps ${STEPS:-5} --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"dtype": "[a-z0-9]*"\|"step_s": [^]]*'
done
done
