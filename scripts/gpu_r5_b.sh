#!/bin/bash
# Metric microbenchmark, headline (5 steps, fit phases), Parquet ingest inside the timed train (10M x 200),
# CSV ingest (2M rows).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u scripts/bench_metric.py > gpurun_out/r5b_bench_metric.log 2>&1 || { tail -20 gpurun_out/r5b_bench_metric.log; exit 1; }
cat gpurun_out/r5b_bench_metric.log
TMOG_FIT_PHASES=1 timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --verbose > gpurun_out/r5b_full.log 2>&1 || { tail -20 gpurun_out/r5b_full.log; exit 1; }
grep -a '^{' gpurun_out/r5b_full.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"best_model": "[A-Za-z]*"\|"fit_phases": {[^}]*}\|"timings": {[^}]*}'
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --verbose --ingest parquet > gpurun_out/r5b_ingest_parquet.log 2>&1 || { tail -20 gpurun_out/r5b_ingest_parquet.log; exit 1; }
grep -a '^{' gpurun_out/r5b_ingest_parquet.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*'
timeout -k 10 400 python3 -u bench.py --rows 2000000 --steps 2 --warmup 1 --verbose --ingest csv > gpurun_out/r5b_ingest_csv.log 2>&1 || { tail -20 gpurun_out/r5b_ingest_csv.log; exit 1; }
grep -a '^{' gpurun_out/r5b_ingest_csv.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*'
