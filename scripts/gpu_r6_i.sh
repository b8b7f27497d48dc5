#!/bin/bash
# Round 6: rocprofv3 kernel statistics of a short default bench run at HEAD (the r6h pass's trace exceeded the
# 64 MiB copy-back, so only the stats CSVs are kept).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -type f ! -name "*stats.csv" -delete
find $O/prof -name "*kernel_stats.csv" -exec head -25 {} \;
grep -a '^{' $O/prof.log | cut -c1-300
