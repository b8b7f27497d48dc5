#!/bin/bash
# Learner lanes A/B (priority on / off, lanes off) after the single-group grower runs on the caller's stream.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-l2}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --verbose > gpurun_out/${T}_${tag}.log 2>&1 || return $?
  grep '^{' gpurun_out/${T}_${tag}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$tag', round(d['value'],4), d['holdout_aupr'], {k: round(v,3) for k,v in d['timings'].items()})"
}
timeout -k 10 300 python -u -m pytest tests/test_concurrent_lanes.py tests/test_tree_engine.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_test.log 2>&1 && tail -n 1 gpurun_out/${T}_test.log && \
run on X=1 && run off TMOG_LEARNER_LANES=1 && run noprio TMOG_LANE_PRIO=0 && run on2 X=1 && run off2 TMOG_LEARNER_LANES=1
