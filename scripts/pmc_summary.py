"""Reduce rocprofv3 CSV outputs (kernel stats + counter passes) to per-kernel totals and derived rates."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
dur = {}
for f in glob.glob(os.path.join(root, "stats", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]))
acc = collections.defaultdict(float)
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"], r["Counter_Name"])] += float(r.get("Counter_Value") or 0)
names = sorted({k for k, _ in acc}, key=lambda n: -dur.get(n, (0, 0))[1])
for n in names:
    calls, ns = dur.get(n, (0, 0.0))
    c = {cn: v for (kn, cn), v in acc.items() if kn == n}
    print(f"== {n[:110]}\n   calls {calls}  total {ns / 1e6:.1f} ms")
    for cn in sorted(c):
        print(f"   {cn:28s} {c[cn]:.4g}")
    if ns > 0:
        if "FETCH_SIZE" in c:
            print(f"   -> fetch {c['FETCH_SIZE'] * 1024 / ns:.1f} GB/s (HBM/MALL side of L2)")
        if "WRITE_SIZE" in c:
            print(f"   -> write {c['WRITE_SIZE'] * 1024 / ns:.1f} GB/s")
    if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
        print(f"   -> L2 hit {c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}")
    if c.get("SQ_WAVE_CYCLES") and c.get("SQ_BUSY_CYCLES"):
        print(f"   -> mean resident waves {c['SQ_WAVE_CYCLES'] / c['SQ_BUSY_CYCLES']:.1f} (per SE-sampled busy cycle)")
    if c.get("SQ_WAIT_INST_LDS") and c.get("SQ_WAVE_CYCLES"):
        print(f"   -> LDS-wait share {c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:.3f}")
    if c.get("SQ_LDS_BANK_CONFLICT") and c.get("SQ_INSTS_LDS"):
        print(f"   -> bank-conflict cycles per LDS instr {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_INSTS_LDS']:.2f}")
