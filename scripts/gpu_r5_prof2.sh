#!/bin/bash
# Kernel statistics: multiclass-text and the headline at bf16 (one timed train each).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-multiclass-text binary-10m}; do
  o=gpurun_out/r5_prof2_${cfg}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$cfg -o run -- python3 -u bench.py --config $cfg --steps 1 --warmup 1 ${BENCH_ARGS} > $o.log 2>&1 || { tail -20 $o.log; exit 1; }
  grep -a '^{' $o.log | grep -o '"value": [0-9.]*'
  S=$(find /tmp/prof_$cfg -name '*kernel_stats.csv' | head -n 1)
  python3 scripts/kstats.py $S 2 40 > $o.kstats.txt || exit 1
  head -25 $o.kstats.txt
  rm -rf /tmp/prof_$cfg
done
