#!/bin/bash
# Per-stream timeline of the XGBoost phase (XGBoost-only selector, warm-up + 1 step, kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
D=/tmp/tr_streams
rm -rf $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --models OpXGBoostClassifier --steps 1 --warmup 1 > gpurun_out/r5s.log 2>&1 || exit $?
T=$(find $D -name '*kernel_trace.csv' | head -n 1)
python3 scripts/stream_timeline.py $T hist_build --last --sample > gpurun_out/r5s_streams.txt || exit $?
cat gpurun_out/r5s_streams.txt
