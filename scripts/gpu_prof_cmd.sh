#!/bin/bash
# rocprofv3 kernel-trace --stats of an arbitrary python command line ($PROG, run from the repo root);
# only the summary CSVs are kept (trace CSVs deleted to stay under the gpurun_out size cap).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_cmd
rm -rf $OUT
cd $GRAFT_REPO_ROOT && timeout -k 10 ${PROF_T:-300} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $PROG > gpurun_out/prof_cmd.log 2>&1; rc=$?
tail -2 gpurun_out/prof_cmd.log
find $OUT -name "*trace*" -delete
exit $rc
