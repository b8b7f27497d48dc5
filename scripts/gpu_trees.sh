#!/bin/bash
# Tree-engine microbenchmarks + kernel-trace profile (summary CSVs only).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/bench_trees.py ${GH_ARGS} > gpurun_out/trees_gh.log 2>&1 || { tail -20 gpurun_out/trees_gh.log; exit 1; }
tail -1 gpurun_out/trees_gh.log
timeout -k 10 300 python benchmarks/bench_trees.py --rf --trees 50 --depth 12 ${RF_ARGS} > gpurun_out/trees_rf.log 2>&1 || { tail -20 gpurun_out/trees_rf.log; exit 1; }
tail -1 gpurun_out/trees_rf.log
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_trees
rm -rf $OUT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_trees.py --rounds 2 ${GH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof_trees.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_trees/**/*kernel_trace.csv", recursive=True)
if f:
    rows = list(csv.DictReader(open(f[0])))
    out = open("gpurun_out/prof_trees/trace_summary.txt", "w")
    for r in rows[:4000]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        out.write(f'{r["Start_Timestamp"]} {d:9.1f}us {r["Kernel_Name"][:60]} grid={r.get("Grid_Size","")}\n')
PY
find $OUT -name "*trace*.csv" -delete
exit $rc
