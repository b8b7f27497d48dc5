#!/bin/bash
# Kernel statistics of the LR objective passes at fp32 and bf16 (LR-only selectors: lr-rf-1m and the headline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-lr-rf-1m binary-10m}; do
for dt in fp32 bf16; do
  o=gpurun_out/r5_prof_lr_${cfg}_$dt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$dt -o run -- python3 -u bench.py --config $cfg --models OpLogisticRegression --dtype $dt --steps 2 --warmup 1 > $o.log 2>&1 || { tail -20 $o.log; exit 1; }
  grep -a '^{' $o.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*'
  S=$(find /tmp/prof_$dt -name '*kernel_stats.csv' | head -n 1)
  python3 scripts/kstats.py $S 3 14 > $o.kstats.txt || exit 1
  head -8 $o.kstats.txt
  rm -rf /tmp/prof_$dt
done
done
