#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/fe_profile.py multiclass-text 1000000 > gpurun_out/r5h_fe_mct.log 2>&1 || { tail -20 gpurun_out/r5h_fe_mct.log; exit 1; }
head -3 gpurun_out/r5h_fe_mct.log
timeout -k 10 300 python3 -u scripts/fe_profile.py binary 10000000 > gpurun_out/r5h_fe_bin.log 2>&1 || { tail -20 gpurun_out/r5h_fe_bin.log; exit 1; }
head -3 gpurun_out/r5h_fe_bin.log
TMOG_INGEST_PROFILE=1 timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --verbose --ingest parquet > gpurun_out/r5h_ingest_parquet.log 2>&1 || { tail -20 gpurun_out/r5h_ingest_parquet.log; exit 1; }
grep -a 'ingest-profile' gpurun_out/r5h_ingest_parquet.log
grep -a '^{' gpurun_out/r5h_ingest_parquet.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*'
