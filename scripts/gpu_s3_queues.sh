#!/bin/bash
# Hardware queues x learner lanes A/B of the headline on one box (GPU_MAX_HW_QUEUES <= 32).
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-q}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --verbose > gpurun_out/${T}_${tag}.log 2>&1 || return $?
  grep '^{' gpurun_out/${T}_${tag}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$tag', round(d['value'],4), d['holdout_aupr'], {k: round(v,3) for k,v in d['timings'].items()})"
}
run q8_on GPU_MAX_HW_QUEUES=8 && run q16_on GPU_MAX_HW_QUEUES=16 && run q16_off GPU_MAX_HW_QUEUES=16 TMOG_LEARNER_LANES=1 && \
run q4_on GPU_MAX_HW_QUEUES=4 && run q8_off GPU_MAX_HW_QUEUES=8 TMOG_LEARNER_LANES=1
