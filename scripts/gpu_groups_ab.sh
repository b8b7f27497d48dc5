#!/bin/bash
# A/B of the tree grower's job-group count (host threads + HIP streams), alternating runs on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gab
export TMPDIR=/tmp
for rep in 1 2; do
  for G in 2 3 6; do
    TMOG_TREE_GROUPS=$G timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/gab/g${G}_r${rep}.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/gab/g${G}_r${rep}.log').read().strip().splitlines()[-1]); print('G=$G rep=$rep', round(d['value'],3), {k: round(v,3) for k,v in d['timings'].items() if k.startswith('Op')})"
  done
done
