#!/bin/bash
# rocprofv3 kernel-trace run of one headline step (extra env passed through: e.g. TMOG_GROW_ON_BASE=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-pb}
mkdir -p gpurun_out
export TMPDIR=/tmp
D=/tmp/prof_$T; rm -rf $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/${T}_prof.log 2>&1 || exit $?
cp $D/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv && python3 scripts/kstats.py gpurun_out/${T}_kernel_stats.csv | head -14
