#!/bin/bash
# Kernel trace of the full headline (warm-up + 1 step): per-kernel totals and idle gaps over the whole step.
# bash scripts/gpu_r4_trace.sh TAG ["extra bench args"]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; EXTRA=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
D=/tmp/tr_$TAG
rm -rf $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 1 --warmup 1 --verbose $EXTRA > gpurun_out/tr_${TAG}.log 2>&1 || exit $?
T=$(find $D -name '*kernel_trace.csv' | head -n 1)
S=$(find $D -name '*kernel_stats.csv' | head -n 1)
python3 scripts/kstats.py $S 2 40 > gpurun_out/tr_${TAG}_kstats.txt || exit $?
python3 scripts/trace_gaps.py $T > gpurun_out/tr_${TAG}_gaps.txt || exit $?
head -45 gpurun_out/tr_${TAG}_kstats.txt; head -12 gpurun_out/tr_${TAG}_gaps.txt
