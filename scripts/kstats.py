"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time (ms per profiled run)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
runs = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 16
tot = sum(int(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6 / runs:.1f} ms per run")
for r in rows[:top]:
    print(f"{int(r['TotalDurationNs']) / 1e6 / runs:9.1f} ms {int(r['Calls']) / runs:8.0f} calls  {r['Name'][:80]}")
