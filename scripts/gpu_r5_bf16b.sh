#!/bin/bash
# bf16 paths after the native pack / exactness kernels and the split-K gradient GEMM: GPU tests, then kernel
# statistics of multiclass-text and the headline, then the two benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_linear_bf16_gpu.py tests/test_sanity_kernels_gpu.py > gpurun_out/r5_bf16b_tests.log 2>&1 || { tail -40 gpurun_out/r5_bf16b_tests.log; exit 1; }
tail -1 gpurun_out/r5_bf16b_tests.log
bash scripts/gpu_r5_prof2.sh || exit 1
for cfg in multiclass-text binary-10m; do
  o=gpurun_out/r5_bf16b_bench_${cfg}.log
  TMOG_FIT_PHASES=1 timeout -k 10 400 python3 -u bench.py --config $cfg --steps 3 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"holdout_error": [0-9.]*\|"step_s": [^]]*'
done
