"""Per-launch size buckets of the tree kernels from a rocprofv3 kernel trace: for each kernel, launches and
total time by workgroup count (log2 buckets), so deep-level (many small nodes) and shallow-level
(few large nodes) costs can be told apart."""
import csv
import glob
import math
import sys
from collections import defaultdict

fn = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
keys = sys.argv[2:] or ["hist_build_kernel<2>", "split_scan_kernel<2>", "partition_fused", "hist_subtract",
                        "zero_segments", "split_reduce"]
acc = {k: defaultdict(lambda: [0, 0]) for k in keys}
with open(fn) as f:
    rd = csv.DictReader(f)
    gk = [c for c in rd.fieldnames if c.startswith("Grid_Size")]
    wk = [c for c in rd.fieldnames if c.startswith("Workgroup_Size")]
    for r in rd:
        n = r["Kernel_Name"]
        for k in keys:
            if k in n:
                g = 1
                for c in gk:
                    g *= max(1, int(r[c]))
                w = 1
                for c in wk:
                    w *= max(1, int(r[c]))
                b = int(math.log2(max(1, g // w)))
                a = acc[k][b]
                a[0] += 1
                a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k in keys:
    tot = sum(v[1] for v in acc[k].values())
    print(f"{k}: {sum(v[0] for v in acc[k].values())} launches, {tot / 1e6:.1f} ms")
    for b in sorted(acc[k]):
        c, t = acc[k][b]
        print(f"   wgs [{2 ** b:6d}, {2 ** (b + 1):6d}): {c:5d} launches  {t / 1e6:8.1f} ms  {t / max(c, 1) / 1e3:7.1f} us/launch")
