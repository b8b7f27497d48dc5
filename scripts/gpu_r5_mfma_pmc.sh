#!/bin/bash
# MFMA counters of the linear objective kernels (fp32 lr_objective_kernel vs bf16 lr_bf16_kernel) at the
# headline's LR shape: one counter pass, kernel-trace only
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/pmc_mf -o pmc -- python3 -u scripts/bench_lr_kernel.py 3300000 329 32 > gpurun_out/r5_mfma_pmc_run.log 2>&1 || { tail -20 gpurun_out/r5_mfma_pmc_run.log; exit 1; }
F=$(find /tmp/pmc_mf -name '*counter_collection.csv' | head -n 1)
python3 - "$F" > gpurun_out/r5_mfma_pmc.txt <<'PY'
import csv, sys, collections, re
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r.get("Kernel_Name", "")
    if "lr_bf16_kernel" in k or "lr_objective_kernel" in k:
        name = re.sub(r"\(anonymous namespace\)::", "", k).split("(")[0].replace("void ", "")[:50]
        agg[name][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(name, r["Counter_Name"])] += 1
for name, c in agg.items():
    n = max(cnt[(name, "SQ_WAVES")], 1)
    busy = c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(c["SQ_BUSY_CYCLES"], 1)
    print(f"{name}: per dispatch MFMA instrs {c['SQ_INSTS_MFMA'] / n:.3g}, VALU instrs {c['SQ_INSTS_VALU'] / n:.3g}, "
          f"waves {c['SQ_WAVES'] / n:.0f}, MFMA-busy / SQ-busy cycles {busy:.3f}  (dispatches {n})")
PY
cat gpurun_out/r5_mfma_pmc.txt
rm -rf /tmp/pmc_mf
