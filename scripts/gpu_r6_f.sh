#!/bin/bash
# Round 6: the GPU CSV reader after the pipeline rework (next chunk copied while the current one parses, one
# deferred check per chunk, dictionaries resolved once at the end): tests, then 10M x 200 ingest inside train()
# with the reader's phase profile, then a kernel-stats pass of the same ingest.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_csv.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
TMOG_INGEST_PROFILE=1 timeout -k 10 700 python3 -u bench.py --ingest csv --ingest-dir /tmp --steps 2 --warmup 1 --verbose > $O/ingest_csv.log 2>&1 || { tail -20 $O/ingest_csv.log; exit 1; }
grep -a "gpu-csv" $O/ingest_csv.log | tail -3
echo "csv $(grep -a '^{' $O/ingest_csv.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*' | tr '\n' ' ')"
