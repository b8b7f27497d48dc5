#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
mkdir -p gpurun_out
bash scripts/gpu_r4_trace.sh $TAG || exit $?
timeout -k 10 300 python -u scripts/pyprof_bench.py gpurun_out/pyprof_${TAG}.txt --steps 1 --warmup 1 --verbose > gpurun_out/pyprof_${TAG}.log 2>&1 || { tail -5 gpurun_out/pyprof_${TAG}.log; exit 1; }
bash scripts/gpu_r4_xgb_ab.sh $TAG 2 "TMOG_XGB_PIPE=2" "TMOG_XGB_PIPE=3" "TMOG_XGB_PIPE=4"
