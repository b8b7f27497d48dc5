#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread tests/test_columnar_ingest.py > gpurun_out/r5d_tests.log 2>&1 || { tail -30 gpurun_out/r5d_tests.log; exit 1; }
tail -1 gpurun_out/r5d_tests.log
TMOG_INGEST_PROFILE=1 timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --verbose --ingest parquet > gpurun_out/r5d_ingest_parquet.log 2>&1 || { tail -20 gpurun_out/r5d_ingest_parquet.log; exit 1; }
grep -a 'ingest-profile' gpurun_out/r5d_ingest_parquet.log
grep -a '^{' gpurun_out/r5d_ingest_parquet.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"DataReadingAndFiltering": [0-9.]*'
D=/tmp/tr_levels
rm -rf $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o run -- python3 bench.py --models OpXGBoostClassifier --steps 1 --warmup 1 > gpurun_out/r5d_levels_run.log 2>&1 || exit $?
T=$(find $D -name '*kernel_trace.csv' | head -n 1)
python3 scripts/xgb_levels.py $T --last > gpurun_out/r5d_xgb_levels.txt || exit $?
cat gpurun_out/r5d_xgb_levels.txt
