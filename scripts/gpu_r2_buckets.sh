#!/bin/bash
# Tree-kernel launch-size buckets and XGBoost busy/idle from one kernel-traced headline step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/buckets
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/bk_trace -o t -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/buckets/run.log 2>&1 || exit 1
python3 scripts/debug/trace_buckets.py /tmp/bk_trace > gpurun_out/buckets/buckets.txt 2>&1
python3 scripts/debug/trace_gaps.py /tmp/bk_trace > gpurun_out/buckets/xgb_busy_idle.txt 2>&1
cat gpurun_out/buckets/*.txt
