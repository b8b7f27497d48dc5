#!/bin/bash
# Host-side profile (cProfile) of the 10M bench restricted to $MODELS, top functions by own time.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m cProfile -o /tmp/bench.prof bench.py --rows ${ROWS:-10000000} --warmup 1 --steps 1 --models ${MODELS:-OpXGBoostClassifier} > gpurun_out/cprof_bench.log 2>&1 || exit $?
python - > gpurun_out/cprof.txt <<'PY'
import pstats
p = pstats.Stats("/tmp/bench.prof")
p.sort_stats("tottime").print_stats(35)
p.sort_stats("cumulative").print_stats(45)
PY
tail -1 gpurun_out/cprof_bench.log | cut -c1-300
