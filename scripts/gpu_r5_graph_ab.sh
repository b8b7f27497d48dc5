#!/bin/bash
# A/B of the hipGraph objective passes (TMOG_LR_GRAPH) on lr-rf-1m and the LR-only headline selector
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for g in 0 1 0 1; do
  o=gpurun_out/r5_graph_ab_$g.log
  TMOG_LR_GRAPH=$g timeout -k 10 300 python3 -u bench.py --config lr-rf-1m --steps 5 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  echo "graph=$g $(grep -a '^{' $o | grep -o '"value": [0-9.]*\|"OpLogisticRegression": [0-9.]*' | tr '\n' ' ')"
done
for g in 0 1; do
  o=gpurun_out/r5_graph_ab_head_$g.log
  TMOG_LR_GRAPH=$g timeout -k 10 300 python3 -u bench.py --models OpLogisticRegression --steps 3 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  echo "head LR-only graph=$g $(grep -a '^{' $o | grep -o '"value": [0-9.]*\|"OpLogisticRegression": [0-9.]*' | tr '\n' ' ')"
done
