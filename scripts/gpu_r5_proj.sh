#!/bin/bash
# Phase breakdown of the headline XGBoost learner, then the 2/4/8-rank projections of the headline (each rank's
# share of the shard schedule timed on this GPU, collectives answered locally).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r5_phases.sh || exit $?
for w in 2 4 8; do
  timeout -k 10 900 python -u scripts/project_schedule.py --world $w --timeout 240 --out gpurun_out/proj$w > gpurun_out/proj$w.log 2>&1 || { tail -5 gpurun_out/proj$w.log; exit 1; }
  tail -1 gpurun_out/proj$w.log
done
