#!/bin/bash
# PMC pass over the LR objective micro-benchmark (kernel-trace + counters only).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/linpmc
rm -rf $OUT
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_linear.py --rows 1000000 --cols 329 --problems 24 --reps 5 > $GRAFT_REPO_ROOT/gpurun_out/linpmc.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob, collections
fs = glob.glob("gpurun_out/linpmc/**/*counter_collection.csv", recursive=True)
out = open("gpurun_out/linpmc_summary.txt", "w")
for f in fs:
    acc = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = (r.get("Kernel_Name", "")[:60], r.get("Counter_Name"))
        acc[k] += float(r.get("Counter_Value", 0) or 0); n[k] += 1
    for k in sorted(acc):
        if "lr_" in k[0]:
            out.write(f"{k[0]:60s} {k[1]:28s} {acc[k]:.4g} (n={n[k]})\n")
PY
find $OUT -name "*.csv" -size +2M -delete
cat gpurun_out/linpmc_summary.txt
exit $rc
