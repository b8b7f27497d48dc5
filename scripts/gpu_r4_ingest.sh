#!/bin/bash
# Ingest inside the timed region: the headline with the table read from a Parquet file by every timed train.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
df -h /tmp /dev/shm > gpurun_out/ingest_df.txt 2>&1
timeout -k 10 200 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_columnar_ingest.py > gpurun_out/ingest_tests.log 2>&1 || { tail -30 gpurun_out/ingest_tests.log; exit 1; }
tail -2 gpurun_out/ingest_tests.log
timeout -k 10 600 python -u bench.py --ingest parquet --steps 2 --warmup 1 --verbose > gpurun_out/ingest_bench.log 2>&1 || { tail -30 gpurun_out/ingest_bench.log; exit 1; }
grep -a '^\[ingest\]' gpurun_out/ingest_bench.log
grep -a '^{' gpurun_out/ingest_bench.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*\|"step_s": \[[^]]*\]'
