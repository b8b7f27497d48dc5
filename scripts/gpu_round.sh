#!/bin/bash
# One GPU session: tests, smoke, short bench. Each GPU step has its own time limit; stop at first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
tail -5 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${BENCH_T:-400} python bench.py --rows ${ROWS:-1000000} --warmup ${WARMUP:-1} --steps 1 --verbose > gpurun_out/bench.log 2>&1; rc=$?
tail -5 gpurun_out/bench.log
exit $rc
