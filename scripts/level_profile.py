"""Per-tree-level breakdown of the tree grower from a rocprofv3 kernel trace:
python scripts/level_profile.py <kernel_trace.csv> [window-substring]

Kernels are grouped by the stream (queue) they ran on; on each stream a level starts at a
``zero_segments_kernel`` launch (one per level and group) and a boosting round ends at a
``boost_epilogue_kernel``, so the depth of a level is its position since the last epilogue. For every
depth it prints the level count, the summed kernel time per kernel family, and the host turnaround: the
idle time on that stream between the end of a level's last kernel and the start of the next level's
first kernel (the per-level result read + host planning + staging copy + launches)."""
import csv
import sys
from collections import defaultdict

FAMILIES = ["hist_build", "pair_scan", "split_scan", "split_reduce", "partition_fused", "zero_segments",
            "hist_subtract", "leaf_collect", "boost_epilogue", "aupr_counts", "level_plan", "copyBuffer"]


def fam(name: str) -> str:
    for f in FAMILIES:
        if f in name:
            return f
    return "other"


def main():
    path = sys.argv[1]
    win = sys.argv[2] if len(sys.argv) > 2 else "hist_build_kernel<2"
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            s = int(r.get("Start_Timestamp") or r.get("BeginNs"))
            e = int(r.get("End_Timestamp") or r.get("EndNs"))
            q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
            rows.append((s, e, name, q))
    rows.sort()
    sel = [i for i, r in enumerate(rows) if win in r[2]]
    if not sel:
        print("no dispatch matches", win)
        return
    lo, hi = rows[sel[0]][0], rows[sel[-1]][1]
    rows = [r for r in rows if lo <= r[0] and r[1] <= hi]
    by_q = defaultdict(list)
    for r in rows:
        by_q[r[3]].append(r)
    tot = defaultdict(lambda: defaultdict(float))   # depth -> family -> ns
    cnt = defaultdict(int)
    turn = defaultdict(list)                          # depth -> host turnaround before that level (ns)
    for q, rs in by_q.items():
        if not any("zero_segments" in r[2] for r in rs):
            continue
        depth = -1
        last_end = None
        for s, e, n, _ in rs:
            f = fam(n)
            if f == "zero_segments":
                depth += 1
                cnt[depth] += 1
                if last_end is not None and depth > 0:
                    turn[depth].append(s - last_end)
            if f == "boost_epilogue":
                depth = -1
                last_end = None
                continue
            if depth >= 0:
                tot[depth][f] += e - s
            last_end = e
    shown = [f for f in FAMILIES if any(tot[d][f] for d in tot)]
    print(f"window {(hi - lo) / 1e6:.1f} ms, streams with levels: "
          f"{sum(1 for q in by_q if any('zero_segments' in r[2] for r in by_q[q]))}")
    print("depth  levels " + " ".join(f"{f[:12]:>12s}" for f in shown) + "   turnaround p50/mean us  total ms")
    gsum = defaultdict(float)
    tsum = 0.0
    for d in sorted(tot):
        t = sorted(turn[d])
        p50 = t[len(t) // 2] / 1e3 if t else 0.0
        mean = sum(t) / len(t) / 1e3 if t else 0.0
        tsum += sum(t)
        for f in shown:
            gsum[f] += tot[d][f]
        print(f"{d:5d} {cnt[d]:7d} " + " ".join(f"{tot[d][f] / 1e6:12.1f}" for f in shown)
              + f"   {p50:9.1f} / {mean:7.1f}   {sum(t) / 1e6:7.1f}")
    print("  all         " + " ".join(f"{gsum[f] / 1e6:12.1f}" for f in shown) + f"   turnaround total {tsum / 1e6:.1f} ms")


if __name__ == "__main__":
    main()
