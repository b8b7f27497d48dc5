#!/bin/bash
# Round-3 check: GPU suite, smoke, headline bench (driver-like step count), one kernel-stats profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r3}
STEPS=${STEPS:-5}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py --steps $STEPS --warmup 2 --verbose > gpurun_out/${TAG}_bench.log 2>&1
rc=$?
tail -n 2 gpurun_out/${TAG}_gputest.log; tail -n 2 gpurun_out/${TAG}_smoke.log; tail -n 1 gpurun_out/${TAG}_bench.log
exit $rc
