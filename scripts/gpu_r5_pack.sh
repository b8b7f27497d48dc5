#!/bin/bash
# bf16 packing kernel: numerics tests that cover it, then the microbench (kernel stats under rocprofv3)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_linear_bf16_gpu.py tests/test_sanity_kernels_gpu.py > gpurun_out/r5_pack_tests.log 2>&1 || { tail -30 gpurun_out/r5_pack_tests.log; exit 1; }
tail -2 gpurun_out/r5_pack_tests.log
timeout -k 10 300 python3 -u scripts/bench_pack.py > gpurun_out/r5_pack_bench.log 2>&1 || { tail -20 gpurun_out/r5_pack_bench.log; exit 1; }
cat gpurun_out/r5_pack_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pk -o pk -- python3 -u scripts/bench_pack.py > gpurun_out/r5_pack_prof.log 2>&1 || { tail -20 gpurun_out/r5_pack_prof.log; exit 1; }
F=$(find /tmp/pk -name '*kernel_stats.csv' | head -n 1)
python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$F')))[:8]: print(f\"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):5d} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:80]}\")
" > gpurun_out/r5_pack_kstats.txt
cat gpurun_out/r5_pack_kstats.txt
rm -rf /tmp/pk
