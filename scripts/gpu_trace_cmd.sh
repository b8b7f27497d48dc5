#!/bin/bash
# rocprofv3 kernel trace of $PROG summarised per (kernel, grid size bucket) -> gpurun_out/trace_summary.txt
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/trace_cmd
rm -rf $OUT
cd $GRAFT_REPO_ROOT && timeout -k 10 ${PROF_T:-300} rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $PROG > gpurun_out/trace_cmd.log 2>&1; rc=$?
python3 - <<'PY'
import csv, glob, collections, math
f = glob.glob("gpurun_out/trace_cmd/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(f[0]))) if f else []
acc = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    name = r.get("Kernel_Name", "")[:60]
    g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) * int(r.get("Grid_Size_Y", 1) or 1)
    wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1)
    blocks = max(1, g // max(wg, 1))
    b = 2 ** int(math.log2(blocks))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    acc[(name, b)][0] += 1
    acc[(name, b)][1] += d
with open("gpurun_out/trace_summary.txt", "w") as o:
    for (k, b), (n, t) in sorted(acc.items(), key=lambda kv: -kv[1][1])[:60]:
        o.write(f"{t/1e3:9.2f} ms {n:6d} calls  blocks~{b:7d}  avg {t/n:8.1f} us  {k}\n")
PY
rm -rf $OUT
exit $rc
