#!/bin/bash
# Kernel trace of the 10M bench, reduced on the box to a busy / idle summary of the XGBoost phase.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=/tmp/trace_out
rm -rf $OUT
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rows ${PROF_ROWS:-10000000} --warmup ${TRACE_WARMUP:-1} --steps 1 --verbose ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/trace_bench.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && for f in "hist_build_kernel<2>" "hist_build_kernel<0>" "lr_objective_kernel"; do echo "== $f"; python3 scripts/debug/trace_gaps.py $OUT --focus "$f" || exit $?; done > gpurun_out/trace_gaps.txt 2>&1 && python3 scripts/debug/trace_timeline.py $OUT > gpurun_out/trace_timeline.txt 2>&1; rc=$?
cat gpurun_out/trace_gaps.txt
exit $rc
