#!/bin/bash
# level planner placement: kernel stats of the headline with the default planner (1024 threads, LDS scratch) and
# with the smallest footprint (256 threads, global scratch)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "base" "small TMOG_PLAN_THREADS=256 TMOG_PLAN_LDS=0"; do
  set -- $cfg
  tag=$1; shift
  env "$@" timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pp_$tag -o pp -- python3 -u bench.py --steps 2 --warmup 1 --verbose > gpurun_out/r5_planab_$tag.log 2>&1 || { tail -20 gpurun_out/r5_planab_$tag.log; exit 1; }
  F=$(find /tmp/pp_$tag -name '*kernel_stats.csv' | head -n 1)
  python3 -c "
import csv
for r in csv.DictReader(open('$F')):
    if any(k in r['Name'] for k in ('level_plan', 'tree_finalize', 'hist_build_kernel<2', 'pair_scan')):
        print(f\"$tag {float(r['AverageNs'])/1e3:8.1f} us avg {int(r['Calls']):6d} calls  {r['Name'][:60]}\")
"
  echo "$tag $(grep -a '^{' gpurun_out/r5_planab_$tag.log | grep -o '"value": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*' | tr '\n' ' ')"
  rm -rf /tmp/pp_$tag
done
