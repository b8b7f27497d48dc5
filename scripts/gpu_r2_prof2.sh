#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TMOG_MEM_TRACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --verbose > gpurun_out/p2_mem.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p2_prof -o p2 -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/p2_prof.log 2>&1
rc=$?
find gpurun_out -name '*trace*.csv' -delete; find gpurun_out -name '*.db' -delete
tail -n 3 gpurun_out/p2_mem.log
exit $rc
