#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TMOG_INGEST_PROFILE=1 timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --verbose --ingest parquet > gpurun_out/r5g_ingest_parquet.log 2>&1 || { tail -20 gpurun_out/r5g_ingest_parquet.log; exit 1; }
grep -a 'ingest-profile' gpurun_out/r5g_ingest_parquet.log
grep -a '^{' gpurun_out/r5g_ingest_parquet.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*'
for w in 2 4 8; do
  timeout -k 10 900 python -u scripts/project_schedule.py --world $w --timeout 240 --out gpurun_out/proj$w > gpurun_out/proj$w.log 2>&1 || { tail -5 gpurun_out/proj$w.log; exit 1; }
  tail -1 gpurun_out/proj$w.log
done
