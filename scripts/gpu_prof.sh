#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench run; only the summary CSVs are kept.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof
rm -rf $OUT
cd /tmp && timeout -k 10 ${PROF_T:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rows ${PROF_ROWS:-1000000} --warmup 0 --steps 1 --verbose ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1; rc=$?
tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof.log
find $OUT -name "*trace*" -delete
ls -la $OUT
exit $rc
