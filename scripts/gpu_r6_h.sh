#!/bin/bash
# Round 6 rehearsal of the round-end GPU tiers at HEAD: the whole GPU suite in one process, smoke(), the default
# 1-GPU bench, and a rocprofv3 kernel-stats pass over a short bench run (copied to profiles/ afterwards).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.log 2>&1 || { tail -40 $O/gpu_suite.log; exit 1; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -a '^{' $O/bench.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
# regression-100m at a 20M training sample with the lane-shared tree budgets (r6e: the GBT batch hit OOM beside
# the random-forest lane)
timeout -k 10 900 python3 -u bench.py --config regression-100m --max-training-sample 20000000 --steps 1 --warmup 1 --verbose > $O/reg100m_20m.log 2>&1 || { tail -30 $O/reg100m_20m.log; exit 1; }
echo "reg100m-20m $(grep -a '^{' $O/reg100m_20m.log | grep -o '"value": [0-9.]*\|"peak_hbm_gb_per_gpu": [0-9.]*' | tr '\n' ' ')"
grep -a -c "OutOfMemory" $O/reg100m_20m.log || true
