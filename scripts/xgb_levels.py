"""Per-depth cost of the device-planned XGBoost levels from a rocprofv3 kernel trace.

python scripts/xgb_levels.py <kernel_trace.csv> [--last]

The profiler runs dispatches one at a time, so durations are exclusive kernel times. Every boosting part issues
from its own host thread: dispatches are grouped by Thread_Id, and inside a thread every level_plan_kernel
starts a new level (level 0 follows boost_prologue / the first plan of a tree). Prints, per depth, the summed
milliseconds of each level kernel over all trees, and the share of each depth in the XGBoost kernel time."""
import csv
import sys
from collections import defaultdict

LEVEL_KERNELS = ("zero_segments", "hist_build", "pair_scan", "split_scan", "partition_fused", "leaf_collect",
                 "level_plan", "hist_subtract")


def short(name):
    for k in LEVEL_KERNELS + ("tree_finalize", "boost_epilogue", "boost_prologue", "aupr_counts"):
        if k in name:
            return k
    return None


def main():
    path = sys.argv[1]
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            k = short(r.get("Kernel_Name") or "")
            if k is None:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r.get("Thread_Id", "0")))
    rows.sort()
    if "--last" in sys.argv and rows:     # the timed step: after the last gap > 200 ms between XGBoost kernels
        start = 0
        for i in range(1, len(rows)):
            if rows[i][0] - rows[i - 1][1] > 200_000_000:
                start = i
        rows = rows[start:]
    by_thread = defaultdict(list)
    for r in rows:
        by_thread[r[3]].append(r)
    depth_cost = defaultdict(lambda: defaultdict(float))
    per_round = defaultdict(float)
    total = 0.0
    for th, rs in by_thread.items():
        d = -1
        for s, e, k, _ in rs:
            dur = (e - s) / 1e6
            total += dur
            if k == "boost_prologue" or k == "tree_finalize" or k == "boost_epilogue" or k == "aupr_counts":
                per_round[k] += dur
                if k == "boost_prologue":
                    d = -1
                continue
            if k == "level_plan":
                d += 1
            depth_cost[max(d, 0)][k] += dur
    print(f"XGBoost kernel time {total:.1f} ms over {len(by_thread)} host threads")
    ks = [k for k in LEVEL_KERNELS if any(k in v for v in depth_cost.values())]
    print("depth " + " ".join(f"{k[:12]:>12}" for k in ks) + "      total  share")
    for d in sorted(depth_cost):
        row = depth_cost[d]
        t = sum(row.values())
        print(f"{d:5d} " + " ".join(f"{row.get(k, 0.0):12.1f}" for k in ks) + f" {t:10.1f} {100 * t / total:5.1f}%")
    print("per round: " + ", ".join(f"{k} {v:.1f}" for k, v in per_round.items()))


if __name__ == "__main__":
    main()
