#!/bin/bash
# Full GPU suite + smoke + headline bench + kernel-stats profile (round-end rehearsal).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-chk}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/${TAG}_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o ${TAG} -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
find gpurun_out -name '*trace*.csv' -delete; find gpurun_out -name '*.db' -delete
tail -n 1 gpurun_out/${TAG}_gputest.log; tail -n 1 gpurun_out/${TAG}_smoke.log; tail -n 1 gpurun_out/${TAG}_bench.log
exit $rc
