"""Per-stream view of a rocprofv3 kernel trace: python scripts/stream_timeline.py <kernel_trace.csv> [key] [--last]

Window: first..last dispatch whose name contains ``key`` (default hist_build); with --last, only the last
contiguous run of such dispatches separated by > 100 ms from the previous (the timed step after the warm-up).
For every queue (HIP stream -> hardware queue) in the window: dispatches, time with a kernel of that queue
running, idle time between its kernels; then the time-weighted number of queues running a kernel at once
and an estimate of the CUs busy (sum over running kernels of min(workgroups, 256) / 256, capped at 1)."""
import csv
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path = args[0]
    key = args[1] if len(args) > 1 else "hist_build"
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or ""
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            q = r.get("Queue_Id") or r.get("Stream_Id") or "0"
            gx = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
            wx = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 1)
            rows.append((s, e, name, q, max(1, gx // max(wx, 1))))
    rows.sort()
    sel = [r for r in rows if key in r[2]]
    if not sel:
        print("no dispatch matches", key)
        return
    if "--last" in sys.argv:
        start = 0
        for i in range(1, len(sel)):
            if sel[i][0] - sel[i - 1][1] > 100_000_000:
                start = i
        sel = sel[start:]
    lo, hi = sel[0][0], sel[-1][1]
    win = [r for r in rows if r[0] >= lo and r[1] <= hi]
    span = hi - lo
    print(f"window {span / 1e6:.2f} ms, {len(win)} dispatches (key {key!r})")
    byq = defaultdict(list)
    for r in win:
        byq[r[3]].append(r)
    print(f"{'queue':>8} {'disp':>7} {'busy ms':>9} {'idle ms':>9} {'busy %':>7}  top kernels (ms)")
    for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        rs.sort()
        busy, cur_s, cur_e = 0, rs[0][0], rs[0][1]
        for s, e, *_ in rs[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        qspan = rs[-1][1] - rs[0][0]
        tot = defaultdict(int)
        for s, e, n, *_ in rs:
            tot[n.split("(")[0].replace("(anonymous namespace)::", "")[:40]] += e - s
        top = ", ".join(f"{n} {v / 1e6:.0f}" for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[:4])
        print(f"{q:>8} {len(rs):7d} {busy / 1e6:9.1f} {(qspan - busy) / 1e6:9.1f} {100 * busy / max(qspan, 1):6.1f}%  {top}")
    # sweep: concurrency and CU estimate
    ev = []
    for s, e, n, q, wg in win:
        ev.append((s, 1, min(wg, 256) / 256.0))
        ev.append((e, -1, min(wg, 256) / 256.0))
    ev.sort(key=lambda t: (t[0], t[1]))
    t_prev, nrun, cu = ev[0][0], 0, 0.0
    hist = defaultdict(int)
    cu_time = 0.0
    for t, d, w in ev:
        dt = t - t_prev
        hist[nrun] += dt
        cu_time += min(cu, 1.0) * dt
        nrun += d
        cu += d * w
        t_prev = t
    print("kernels running at once (share of window):",
          ", ".join(f"{k}: {100 * v / span:.1f}%" for k, v in sorted(hist.items())))
    print(f"estimated CU occupancy (workgroups vs 256 CUs, capped): {100 * cu_time / span:.1f}% of the window")




def sample(path, key="hist_build", n=40):
    """The middle ``n`` dispatches of the busiest queue in the window: gap before each, duration, name."""
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name") or "",
                         r.get("Queue_Id") or "0"))
    rows.sort()
    sel = [r for r in rows if key in r[2]]
    lo, hi = sel[0][0], sel[-1][1]
    byq = defaultdict(list)
    for r in rows:
        if lo <= r[0] and r[1] <= hi:
            byq[r[3]].append(r)
    q, rs = max(byq.items(), key=lambda kv: len(kv[1]))
    m = len(rs) // 2
    print(f"queue {q}: dispatches {m}..{m + n}")
    prev = rs[m - 1][1]
    for s, e, name, _ in rs[m:m + n]:
        print(f"  gap {(s - prev) / 1e3:8.1f} us  dur {(e - s) / 1e3:8.1f} us  {name.split('(')[0][-50:]}")
        prev = e


if __name__ == "__main__":
    main()
    if "--sample" in sys.argv:
        sample(sys.argv[1], [a for a in sys.argv[2:] if not a.startswith("--")][0] if len(
            [a for a in sys.argv[2:] if not a.startswith("--")]) else "hist_build")
