"""Timeline of a rocprofv3 kernel trace: per time bin, GPU busy fraction and the kernels that filled it."""
import argparse
import csv
import glob
import re

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--bin-ms", type=float, default=100.0)
a = ap.parse_args()
fn = glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True)[0]
iv, names = [], []
with open(fn) as f:
    for r in csv.DictReader(f):
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        n = re.sub(r"^void ", "", r["Kernel_Name"])
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = re.sub(r"<.*", "", n).split("(")[0]
        names.append(n[-40:])
iv = np.array(iv, dtype=np.int64)
t0 = iv[:, 0].min()
iv = iv - t0
W = int(a.bin_ms * 1e6)
nb = int(iv[:, 1].max() // W) + 1
busy = np.zeros(nb)
top = [dict() for _ in range(nb)]
order = np.argsort(iv[:, 0])
cs, ce = None, None
merged = []
for i in order:
    s, e = iv[i]
    if cs is None or s > ce:
        if cs is not None:
            merged.append((cs, ce))
        cs, ce = s, e
    else:
        ce = max(ce, e)
    b0, b1 = s // W, e // W
    for b in range(b0, b1 + 1):
        ov = min(e, (b + 1) * W) - max(s, b * W)
        if ov > 0:
            top[b][names[i]] = top[b].get(names[i], 0) + ov
merged.append((cs, ce))
for s, e in merged:
    for b in range(s // W, e // W + 1):
        ov = min(e, (b + 1) * W) - max(s, b * W)
        if ov > 0:
            busy[b] += ov
print(f"trace span {iv[:, 1].max() / 1e9:.3f} s, busy {busy.sum() / 1e9:.3f} s")
for b in range(nb):
    t = sorted(top[b].items(), key=lambda x: -x[1])[:3]
    desc = ", ".join(f"{k} {v / 1e6:.0f}" for k, v in t)
    print(f"{b * a.bin_ms / 1000:7.2f}s busy {100 * busy[b] / W:5.1f}%  {desc}")
