#!/bin/bash
# Per-level tree-grower breakdown (scripts/level_profile.py) + occupancy of the XGBoost window from a kernel
# trace of the XGBoost-only selector (warm-up + 1 step); bulky trace kept in /tmp on the box.
# bash scripts/gpu_r4_levels.sh TAG ["extra bench args"]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; EXTRA=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
D=/tmp/lv_$TAG
rm -rf $D
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --models OpXGBoostClassifier --steps 1 --warmup 1 --verbose $EXTRA > gpurun_out/lv_${TAG}.log 2>&1 || exit $?
T=$(ls $D/run_kernel_trace.csv 2>/dev/null || find $D -name '*kernel_trace.csv' | head -n 1)
head -c 600 $T > gpurun_out/lv_${TAG}_header.txt
python3 scripts/trace_gaps.py $T "hist_build_kernel<2" > gpurun_out/lv_${TAG}_gaps.txt || exit $?
head -40 gpurun_out/lv_${TAG}_gaps.txt
python3 scripts/level_profile.py $T > gpurun_out/lv_${TAG}_levels.txt 2>&1 || echo "level_profile failed"
grep '^{' gpurun_out/lv_${TAG}.log | tail -c 400
