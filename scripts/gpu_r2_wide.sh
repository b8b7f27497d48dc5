#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py tests/test_tree_capacity.py tests/test_learner_parallel.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/w_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/w_bench.log 2>&1 && \
TMOG_HIST_WIDE=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/w_bench_off.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/w_prof -o w -- python3 bench.py --steps 1 --warmup 0 > gpurun_out/w_prof.log 2>&1
rc=$?
find gpurun_out -name '*trace*.csv' -delete; find gpurun_out -name '*.db' -delete
tail -n 4 gpurun_out/w_test.log; tail -n 1 gpurun_out/w_bench.log gpurun_out/w_bench_off.log
exit $rc
