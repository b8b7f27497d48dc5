#!/bin/bash
# Summarise the outputs of gpu_iter.sh.
cd "$(dirname "$0")/../.."
tail -3 gpurun_out/iter_tests.log
python - <<'PY'
import csv, json
rows = list(csv.DictReader(open("gpurun_out/prof/run_kernel_stats.csv")))
print("kernel total %.3f s" % (sum(float(r["TotalDurationNs"]) for r in rows) / 1e9))
for r in rows[:8]:
    print("  %-55s %6s %.3f s" % (r["Name"][:55], r["Calls"], float(r["TotalDurationNs"]) / 1e9))
for f in ("gpurun_out/ab_a.log", "gpurun_out/ab_b.log"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"], 3), {k: round(v, 3) for k, v in d["timings"].items()})
PY
