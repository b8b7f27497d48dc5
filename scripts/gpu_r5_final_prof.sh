#!/bin/bash
# kernel statistics of the headline train at the end of round 5 (1 warm-up + 2 timed steps under rocprofv3)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fp -o fp -- python3 -u bench.py --steps 2 --warmup 1 > gpurun_out/r5_final_prof_run.log 2>&1 || { tail -20 gpurun_out/r5_final_prof_run.log; exit 1; }
F=$(find /tmp/fp -name '*kernel_stats.csv' | head -n 1)
python3 -c "
import csv
rows = list(csv.DictReader(open('$F')))
tot = sum(float(r['TotalDurationNs']) for r in rows) / 3e6
print(f'total kernel time {tot:.1f} ms per train (3 trains: 1 warm-up + 2 timed; concurrent lanes, durations include sharing)')
for r in rows[:30]: print(f\"{float(r['TotalDurationNs'])/3e6:9.1f} ms/train {int(r['Calls'])//3:6d} calls/train {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}\")
" > gpurun_out/r5_final_kernel_stats.txt
head -12 gpurun_out/r5_final_kernel_stats.txt
rm -rf /tmp/fp
