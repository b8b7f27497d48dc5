#!/bin/bash
# A/B of an env switch on the headline bench (same box): GPU tree tests, then bench with $AB_VAR=1 and =0.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r3ab}
VAR=${AB_VAR:-TMOG_GH_STAGE}
STEPS=${STEPS:-5}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_gputest.log 2>&1 && \
env $VAR=1 timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 2 --verbose > gpurun_out/${TAG}_on.log 2>&1 && \
env $VAR=0 timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 2 --verbose > gpurun_out/${TAG}_off.log 2>&1
rc=$?
tail -n 2 gpurun_out/${TAG}_gputest.log; tail -c 600 gpurun_out/${TAG}_on.log; echo; tail -c 600 gpurun_out/${TAG}_off.log
exit $rc
