#!/bin/bash
# 8-rank projection of the headline (each rank's share timed on this one GPU, collectives answered locally),
# then a kernel trace of the multiclass-text config and an LR-only multiclass-text run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u scripts/project_schedule.py --world 8 --timeout 240 --out gpurun_out/proj8 || exit $?
timeout -k 10 200 python -u bench.py --config multiclass-text --models OpLogisticRegression --steps 3 --warmup 1 --verbose > gpurun_out/mct_lr.log 2>&1 || exit $?
grep -a '^{' gpurun_out/mct_lr.log | grep -o '"value": [0-9.]*\|"timings": {[^}]*}'
bash scripts/gpu_r4_trace.sh mct "--config multiclass-text"
