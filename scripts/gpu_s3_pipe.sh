#!/bin/bash
# XGBoost boosting parts (TMOG_XGB_PIPE: host threads / streams over the 6 problems) A/B on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-pipe}
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --verbose > gpurun_out/${T}_${tag}.log 2>&1 || return $?
  grep '^{' gpurun_out/${T}_${tag}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$tag', round(d['value'],4), d['holdout_aupr'], {k: round(v,3) for k,v in d['timings'].items()})"
}
run p2 TMOG_XGB_PIPE=2 && run p3 TMOG_XGB_PIPE=3 && run p6 TMOG_XGB_PIPE=6 && run p2b TMOG_XGB_PIPE=2 && run p3b TMOG_XGB_PIPE=3
