#!/bin/bash
# bf16 linear objective: numerics tests, then the lr-rf-1m config at fp32 and at bf16 (same box), with
# per-phase fit times.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_linear_bf16_gpu.py > gpurun_out/r5_bf16_tests.log 2>&1 || { tail -40 gpurun_out/r5_bf16_tests.log; exit 1; }
tail -3 gpurun_out/r5_bf16_tests.log
for dt in fp32 bf16; do
  TMOG_FIT_PHASES=1 timeout -k 10 300 python3 -u bench.py --config lr-rf-1m --dtype $dt --steps 3 --warmup 1 --verbose > gpurun_out/r5_lrrf_$dt.log 2>&1 || { tail -20 gpurun_out/r5_lrrf_$dt.log; exit 1; }
  grep -a '^{' gpurun_out/r5_lrrf_$dt.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"dtype": "[a-z0-9]*"\|"fit_phases": {[^}]*}'
done
