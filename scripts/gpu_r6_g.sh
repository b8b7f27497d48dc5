#!/bin/bash
# Round 6: hardware-queue A/B for the XGBoost lane. The side-stream pool is sized to the process's hardware
# queues (ops/streams.py: GPU_MAX_HW_QUEUES = 4 -> 3 side streams), which caps the XGBoost lane at 3 concurrent
# boosting parts. Here: 8 hardware queues with 5 side streams (4 parts), 7 side streams with 6 parts (one per CV
# job), vs the default, alternating on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
run() {   # tag hwq side pipe
  GPU_MAX_HW_QUEUES=$2 TMOG_SIDE_STREAMS=$3 TMOG_XGB_PIPE=$4 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --verbose > $O/$1.log 2>&1 || { tail -20 $O/$1.log; exit 1; }
  echo "$1 $(grep -a '^{' $O/$1.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*\|"step_s": [^]]*' | tr '\n' ' ')"
}
run base_1 4 3 4 && run q8s5_1 8 5 4 && run q8s7p6_1 8 7 6 && run base_2 4 3 4 && run q8s5_2 8 5 4 && run q8s7p6_2 8 7 6
