#!/bin/bash
# bf16 vs fp32 objective passes at the headline LR shape, then HBM bytes fetched per kernel (TCC FETCH_SIZE; one TCC block per pass)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc_lr -o pmc -- python3 -u scripts/bench_lr_kernel.py 3300000 329 32 > gpurun_out/r5_lr_kernel_pmc_run.log 2>&1 || { tail -20 gpurun_out/r5_lr_kernel_pmc_run.log; exit 1; }
F=$(find /tmp/pmc_lr -name '*counter_collection.csv' | head -n 1)
python3 - "$F" > gpurun_out/r5_lr_kernel_pmc.txt <<'PY'
import csv, sys, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Kernel_Name", "")
    for key in ("lr_bf16_kernel", "lr_objective_kernel"):
        if key in k:
            name = re.sub(r"\(anonymous namespace\)::", "", k).split("(")[0].replace("void ", "")[:60]
            agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[(name, r["Counter_Name"])] += 1
for name, c in agg.items():
    n = max(cnt[(name, "FETCH_SIZE")], 1)
    print(f"{name}: per dispatch FETCH {c['FETCH_SIZE'] / n * 1024 / 1e9:.3f} GB (counter in KiB)   (dispatches {n})")
PY
cat gpurun_out/r5_lr_kernel_pmc.txt
cp "$F" gpurun_out/r5_lr_kernel_pmc_counters.csv; rm -rf /tmp/pmc_lr
