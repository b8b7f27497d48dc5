#!/bin/bash
# A/B of the 10M bench under two environment settings (A = default, B = $AB_ENV), 2 timed steps each.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${BENCH_T:-400} python bench.py --rows ${ROWS:-10000000} --warmup 1 --steps 2 --verbose > gpurun_out/ab_a.log 2>&1 || exit $?
tail -1 gpurun_out/ab_a.log | cut -c1-200
env $AB_ENV timeout -k 10 ${BENCH_T:-400} python bench.py --rows ${ROWS:-10000000} --warmup 1 --steps 2 --verbose > gpurun_out/ab_b.log 2>&1 || exit $?
tail -1 gpurun_out/ab_b.log | cut -c1-200
