#!/bin/bash
# segmented AuPR early-stopping kernel: its test + tree/boosting GPU tests, kernel stats of the XGBoost-only
# selector, then the headline
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_aupr_suite.log 2>&1 || { tail -40 gpurun_out/r5_aupr_suite.log; exit 1; }
tail -1 gpurun_out/r5_aupr_suite.log
timeout -k 10 120 python3 -u -c "
import torch
from transmogrifai_amd.evaluators.metrics import binned_aupr_from_counts
h = torch.randint(0, 4, (2, 2, 1 << 16), dtype=torch.int32, device='cuda')
for _ in range(3): binned_aupr_from_counts(h)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(50): binned_aupr_from_counts(h)
b.record(); torch.cuda.synchronize()
print(f'binned_aupr_from_counts 2 x 65536 bins: {a.elapsed_time(b) / 50 * 1e3:.1f} us per call (kernel + wrapper)')
" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r5_aupr_micro.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ak -o ak -- python3 -u bench.py --models OpXGBoostClassifier --steps 1 --warmup 1 > gpurun_out/r5_aupr_prof.log 2>&1 || { tail -20 gpurun_out/r5_aupr_prof.log; exit 1; }
F=$(find /tmp/ak -name '*kernel_stats.csv' | head -n 1)
python3 -c "
import csv
for r in list(csv.DictReader(open('$F')))[:16]: print(f\"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}\")
" > gpurun_out/r5_aupr_kstats.txt
grep -a "aupr_counts" gpurun_out/r5_aupr_kstats.txt || true
rm -rf /tmp/ak
o=gpurun_out/r5_aupr_bench.log
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
echo "headline $(grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*' | tr '\n' ' ')"
