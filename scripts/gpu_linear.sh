#!/bin/bash
# Linear objective micro-benchmark + rocprofv3 kernel stats of it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python benchmarks/bench_linear.py ${LIN_ARGS} > gpurun_out/linear.log 2>&1 || { tail -20 gpurun_out/linear.log; exit 1; }
tail -1 gpurun_out/linear.log
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_linear
rm -rf $OUT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/bench_linear.py --reps 5 ${LIN_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof_linear.log 2>&1; rc=$?
find $OUT -name "*trace*" -delete
exit $rc
