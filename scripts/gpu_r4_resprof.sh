#!/bin/bash
# Resident-grower tests, then the planner phase profile: bash scripts/gpu_r4_resprof.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_tree_resident_gpu.py > gpurun_out/t_${TAG}.log 2>&1 || { tail -30 gpurun_out/t_${TAG}.log; exit 1; }
tail -3 gpurun_out/t_${TAG}.log
bash scripts/gpu_r4_planprof.sh $TAG
