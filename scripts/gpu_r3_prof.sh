#!/bin/bash
# rocprofv3 kernel stats (+ an occupancy/gap summary of the kernel trace) of one bench run, with the bulky
# trace kept in /tmp on the box: bash scripts/gpu_r3_prof.sh TAG "<bench args>" [trace-window-substring]
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; ARGS=$2; WIN=$3
mkdir -p gpurun_out
export TMPDIR=/tmp
D=/tmp/prof_$TAG
rm -rf $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}.log 2>&1 || exit $?
cp $D/run_kernel_stats.csv gpurun_out/prof_${TAG}_kernel_stats.csv || exit $?
python3 scripts/trace_gaps.py $D/run_kernel_trace.csv > gpurun_out/prof_${TAG}_gaps_all.txt || exit $?
if [ -n "$WIN" ]; then
  python3 scripts/trace_gaps.py $D/run_kernel_trace.csv $WIN > gpurun_out/prof_${TAG}_gaps_win.txt || exit $?
  head -12 gpurun_out/prof_${TAG}_gaps_win.txt
fi
grep '^{' gpurun_out/prof_${TAG}.log | tail -c 600
