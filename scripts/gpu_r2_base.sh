#!/bin/bash
# Round-2 baseline on 1 MI355X: GPU tests, smoke, default bench, kernel-stats profile of the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r2b_gputest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2b_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/r2b_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2b_prof -o r2b -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/r2b_prof.log 2>&1
rc=$?
find gpurun_out -size +2M -ls
find gpurun_out -size +2M -delete
find gpurun_out -type f | head -50
du -sh gpurun_out
exit $rc
