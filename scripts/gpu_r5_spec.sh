#!/bin/bash
# Line search with the first trial's gradient from the same pass (TMOG_OWLQN_SPEC), LR-only headline selector.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for sp in 0 1; do
  o=gpurun_out/r5_spec_$sp
  TMOG_OWLQN_SPEC=$sp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$sp -o run -- python3 -u bench.py --models OpLogisticRegression --steps 2 --warmup 1 > $o.log 2>&1 || { tail -20 $o.log; exit 1; }
  grep -a '^{' $o.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*'
  S=$(find /tmp/prof_$sp -name '*kernel_stats.csv' | head -n 1)
  python3 scripts/kstats.py $S 3 6 > $o.kstats.txt || exit 1
  head -4 $o.kstats.txt
  rm -rf /tmp/prof_$sp
done
for sp in 0 1; do
  TMOG_OWLQN_SPEC=$sp timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 > gpurun_out/r5_spec_head_$sp.log 2>&1 || exit 1
  grep -a '^{' gpurun_out/r5_spec_head_$sp.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*'
done
