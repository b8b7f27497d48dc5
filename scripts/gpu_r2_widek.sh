#!/bin/bash
# Separate wide-load histogram kernel: tree parity tests, then kernel stats of one headline step at
# TMOG_HIST_WIDE_OCC=6 (no spills) and 7 (LDS-limited occupancy, 2 spilled VGPRs).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py tests/test_tree_capacity.py tests/test_gpu_kernels.py tests/test_learner_parallel.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/wk_test.log 2>&1 || { tail -40 gpurun_out/wk_test.log; exit 1; }
tail -2 gpurun_out/wk_test.log
for occ in 6 7; do
  TMOG_HIST_WIDE_OCC=$occ timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wk$occ -o w -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/wk_prof$occ.log 2>&1 || exit 1
done
find gpurun_out -name '*trace*.csv' -delete; find gpurun_out -name '*.db' -delete
for occ in 6 7; do python3 - gpurun_out/wk$occ <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:6]:
    print(sys.argv[1], r["Name"][:50], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 1))
PY
done
