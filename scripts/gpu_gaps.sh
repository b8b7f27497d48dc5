#!/bin/bash
# Busy / idle of the XGBoost phase from a kernel trace of one headline step (summary only kept).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gaps
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/gaps_trace -o t -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/gaps/run.log 2>&1 || exit 1
python3 scripts/debug/trace_gaps.py /tmp/gaps_trace > gpurun_out/gaps/xgb_busy_idle.txt 2>&1
python3 scripts/debug/trace_gaps.py /tmp/gaps_trace --focus lr_objective > gpurun_out/gaps/lr_busy_idle.txt 2>&1
python3 scripts/debug/trace_gaps.py /tmp/gaps_trace --focus "hist_build_kernel<0>" > gpurun_out/gaps/rf_busy_idle.txt 2>&1
cat gpurun_out/gaps/*.txt
