#!/bin/bash
# regression-100m with a 20M-row training sample (tree learners above 2^24 rows), default lanes;
# then (if it passed) the lane-priority A/B (scripts/gpu_r4_prio.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 540 python -u bench.py --config regression-100m --max-training-sample 20000000 --steps 1 --warmup 1 --verbose > gpurun_out/reg20m_b.log 2>&1
rc=$?
grep -a '^{' gpurun_out/reg20m_b.log | grep -o '"value": [0-9.]*\|"holdout_[a-z]*": [0-9.e-]*\|"timings": {[^}]*}\|"peak_hbm_gb_per_gpu": [0-9.]*'
[ $rc -ne 0 ] && { tail -30 gpurun_out/reg20m_b.log; exit $rc; }
bash scripts/gpu_r4_prio.sh a 4
