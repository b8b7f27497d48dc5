#!/bin/bash
# SanityChecker [X | y] single gather: GPU suite, then multiclass-text and headline benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_sc_suite.log 2>&1 || { tail -40 gpurun_out/r5_sc_suite.log; exit 1; }
tail -1 gpurun_out/r5_sc_suite.log
for cfg in multiclass-text binary-10m; do
  o=gpurun_out/r5_sc_bench_${cfg}.log
  timeout -k 10 400 python3 -u bench.py --config $cfg --steps 5 --warmup 1 --verbose > $o 2>&1 || { tail -20 $o; exit 1; }
  echo "$cfg $(grep -a '^{' $o | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"holdout_error": [0-9.]*\|"FeatureEngineering": [0-9.]*\|"fit:SanityChecker[^,]*' | tr '\n' ' ')"
done
