#!/bin/bash
# One kernel-traced headline step (after one warm-up step); the trace is kept gzipped for host analysis.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trace
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o t -- python3 bench.py --steps 1 --warmup 1 ${BENCH_ARGS} > gpurun_out/trace/run.log 2>&1 || exit 1
f=$(find /tmp/kt -name '*kernel_trace.csv' | head -n 1)
python3 - "$f" <<'PY'
import csv, gzip, sys
keep = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Workgroup_Size_X", "Stream_Id", "Queue_Id"]
with open(sys.argv[1]) as f, gzip.open("gpurun_out/trace/kernel_trace.csv.gz", "wt") as o:
    rd = csv.DictReader(f)
    ks = [k for k in keep if k in rd.fieldnames]
    w = csv.writer(o)
    w.writerow(ks)
    for r in rd:
        w.writerow([r[k] for k in ks])
PY
ls -la gpurun_out/trace
