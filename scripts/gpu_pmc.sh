#!/bin/bash
# PMC counters for the tree microbenchmark (kernel-trace + pmc only, no sys/runtime trace).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
rm -rf $OUT
if [ -n "$LIST" ]; then timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_list.txt 2>&1; fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM} --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/${PMC_PROG:-benchmarks/bench_trees.py --rounds 1} ${GH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/pmc.log 2>&1; rc=$?
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob, collections
fs = glob.glob("gpurun_out/pmc/**/*counter_collection.csv", recursive=True)
out = open("gpurun_out/pmc_summary.txt", "w")
for f in fs:
    acc = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = (r.get("Kernel_Name", "")[:50], r.get("Counter_Name"))
        acc[k] += float(r.get("Counter_Value", 0) or 0)
        n[k] += 1
    for k in sorted(acc):
        out.write(f"{k[0]:50s} {k[1]:28s} {acc[k]:.4g} (n={n[k]})\n")
PY
find $OUT -name "*.csv" -size +2M -delete
exit $rc
