#!/bin/bash
# Host-side cProfile of one bench run on the GPU (where does wall-clock go besides kernels).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${PROF_T:-600} python -m cProfile -o gpurun_out/bench.prof bench.py --rows ${PROF_ROWS:-1000000} --warmup 0 --steps 1 --verbose ${BENCH_ARGS} > gpurun_out/pyprof.log 2>&1; rc=$?
tail -2 gpurun_out/pyprof.log
python - <<'PY' > gpurun_out/pyprof.txt
import pstats
p = pstats.Stats("gpurun_out/bench.prof")
p.sort_stats("cumulative").print_stats(70)
p.sort_stats("tottime").print_stats(40)
PY
exit $rc
