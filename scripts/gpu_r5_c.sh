#!/bin/bash
# Ingest inside the timed train (Parquet 10M x 200, CSV 2M), then more hardware queues / boosting parts A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --verbose --ingest parquet > gpurun_out/r5c_ingest_parquet.log 2>&1 || { tail -20 gpurun_out/r5c_ingest_parquet.log; exit 1; }
grep -a '^{' gpurun_out/r5c_ingest_parquet.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*'
timeout -k 10 400 python3 -u bench.py --rows 2000000 --steps 2 --warmup 1 --verbose --ingest csv > gpurun_out/r5c_ingest_csv.log 2>&1 || { tail -20 gpurun_out/r5c_ingest_csv.log; exit 1; }
grep -a '^{' gpurun_out/r5c_ingest_csv.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*'
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 4 --warmup 1 --verbose > gpurun_out/r5c_q_$tag.log 2>&1 || { tail -20 gpurun_out/r5c_q_$tag.log; return 1; }
  echo "$tag $(grep -a '^{' gpurun_out/r5c_q_$tag.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*' | tr '\n' ' ')"
}
run base || exit 1
run q8p6 GPU_MAX_HW_QUEUES=8 TMOG_SIDE_STREAMS=7 TMOG_XGB_PIPE=6 || exit 1
run q8p6l3 GPU_MAX_HW_QUEUES=8 TMOG_SIDE_STREAMS=7 TMOG_XGB_PIPE=6 TMOG_LEARNER_LANES=3 || exit 1
run q6p4 GPU_MAX_HW_QUEUES=6 TMOG_SIDE_STREAMS=5 TMOG_XGB_PIPE=4 || exit 1
run base2 || exit 1
