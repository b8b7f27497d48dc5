"""GPU occupancy of a rocprofv3 kernel trace: python scripts/trace_gaps.py <kernel_trace.csv> [name-substring ...]

Prints the traced span, the time at least one kernel was running (union of the dispatch intervals over
all queues), the idle gaps by size, and per-kernel totals. With name substrings, the window is cut to
the first..last dispatch whose name contains any of them (e.g. the XGBoost phase: hist_build)."""
import csv
import sys
from collections import defaultdict


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    rows = []
    with open(path, newline="") as f:
        rd = csv.DictReader(f)
        for r in rd:
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            s = int(r.get("Start_Timestamp") or r.get("BeginNs"))
            e = int(r.get("End_Timestamp") or r.get("EndNs"))
            gx = int(r.get("Grid_Size_X") or r.get("Grid_Size") or r.get("grd") or 0)
            wx = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or r.get("wgr") or 1)
            rows.append((s, e, name, max(1, gx // max(wx, 1))))
    rows.sort()
    if keys:
        sel = [i for i, (_, _, n, _) in enumerate(rows) if any(k in n for k in keys)]
        if not sel:
            print("no dispatch matches", keys)
            return
        lo, hi = rows[sel[0]][0], rows[sel[-1]][1]
        rows = [r for r in rows if r[0] >= lo and r[1] <= hi]
    span = rows[-1][1] - rows[0][0]
    busy = 0
    cur_s, cur_e = rows[0][0], rows[0][1]
    gaps = []
    for s, e, _, _ in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"dispatches {len(rows)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f} %)")
    edges = [0, 5_000, 20_000, 50_000, 100_000, 250_000, 1_000_000, 10_000_000, 1 << 62]
    for a, b in zip(edges, edges[1:]):
        g = [x for x in gaps if a <= x < b]
        print(f"  gaps [{a / 1e3:>8.0f}, {b / 1e3:>8.0f}) us: n={len(g):6d}  total {sum(g) / 1e6:8.2f} ms")
    tot = defaultdict(list)
    wgs = defaultdict(list)
    for s, e, n, w in rows:
        tot[_short(n)].append(e - s)
        wgs[_short(n)].append((w, e - s))
    print("  total ms   calls  p50 us  p90 us  max us | share of time in calls <20us, 20-100us, 100-500us, >500us")
    for k, d in sorted(tot.items(), key=lambda kv: -sum(kv[1]))[:25]:
        d = sorted(d)
        t = sum(d)
        q = lambda f: d[min(len(d) - 1, int(f * len(d)))] / 1e3
        sh = [sum(x for x in d if a <= x < b) / max(t, 1) for a, b in
              ((0, 20_000), (20_000, 100_000), (100_000, 500_000), (500_000, 1 << 62))]
        print(f"  {t / 1e6:8.2f} {len(d):7d} {q(0.5):7.1f} {q(0.9):7.1f} {d[-1] / 1e3:7.0f} | "
              + " ".join(f"{100 * x:5.1f}%" for x in sh) + f"  {k}")
    # launch size (workgroups) of the heaviest kernels: is the time in under-filled launches?
    wb = [1, 65, 257, 1025, 4097, 16385, 1 << 40]
    print("  workgroups per launch of the top kernels: [lo, hi) n / total ms / mean us")
    for k, d in sorted(tot.items(), key=lambda kv: -sum(kv[1]))[:8]:
        parts = []
        for a, b in zip(wb, wb[1:]):
            x = [t for w, t in wgs[k] if a <= w < b]
            if x:
                parts.append(f"[{a},{b if b < 1 << 40 else 'inf'}) {len(x)}/{sum(x) / 1e6:.1f}/{sum(x) / len(x) / 1e3:.0f}")
        print(f"    {k[:48]:48s} " + "  ".join(parts))


def _short(n: str) -> str:
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    depth, out = 0, []
    for ch in n:                      # drop the argument list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:100]


if __name__ == "__main__":
    main()
