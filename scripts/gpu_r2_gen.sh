#!/bin/bash
# Histogram kernel without the byte-gather path for CSR / wide-only launches: tree parity tests, kernel
# stats of one warmed headline step, and the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py tests/test_tree_capacity.py tests/test_gpu_kernels.py tests/test_learner_parallel.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/g_test.log 2>&1 || { tail -40 gpurun_out/g_test.log; exit 1; }
tail -2 gpurun_out/g_test.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gk -o w -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/g_prof.log 2>&1 || exit 1
find gpurun_out -name '*trace*.csv' -delete; find gpurun_out -name '*.db' -delete
python3 - gpurun_out/gk <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r["Name"][:50], r["Calls"], round(float(r["TotalDurationNs"]) / 2e6, 1), "ms/step")
PY
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/g_bench.log 2>&1
tail -n 1 gpurun_out/g_bench.log
