"""GPU busy / idle analysis of a rocprofv3 kernel trace (run_kernel_trace.csv).

Reports, for the window spanned by kernels whose name contains --focus (default: the XGBoost
histogram kernel), the union of kernel intervals (GPU busy), the idle time, and the idle-gap histogram."""
import argparse
import csv
import glob

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--focus", default="hist_build_kernel<2>")
a = ap.parse_args()
fn = glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True)[0]
iv, names = [], []
with open(fn) as f:
    for r in csv.DictReader(f):
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        names.append(r["Kernel_Name"])
iv = np.array(iv, dtype=np.int64)
foc = np.array([a.focus in n for n in names])
lo, hi = iv[foc, 0].min(), iv[foc, 1].max()
m = (iv[:, 1] >= lo) & (iv[:, 0] <= hi)
w = iv[m]
w = w[np.argsort(w[:, 0])]
busy, gaps = 0, []
cs, ce = w[0]
for s, e in w[1:]:
    if s > ce:
        busy += ce - cs
        gaps.append(s - ce)
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
gaps = np.array(gaps)
print(f"window {(hi - lo) / 1e9:.3f} s  busy {busy / 1e9:.3f} s  idle {(hi - lo - busy) / 1e9:.3f} s  "
      f"kernels {int(m.sum())}")
for t in (5e3, 2e4, 1e5, 1e6):
    sel = gaps >= t
    print(f"  gaps >= {t / 1e3:.0f} us: {int(sel.sum())} totalling {gaps[sel].sum() / 1e9:.3f} s")
tot = {}
for (s, e), n, k in zip(iv, names, m):
    if k:
        key = n.split("(")[0][-50:]
        tot[key] = tot.get(key, 0) + (e - s)
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:10]:
    print(f"  {k:50s} {v / 1e9:.3f} s")
