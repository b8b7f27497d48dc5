#!/bin/bash
# Pipelined XGBoost parts: parity tests, then the headline with TMOG_XGB_PIPE=2 (default) and 1 (off).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k xgb -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/p_test.log 2>&1 || { tail -40 gpurun_out/p_test.log; exit 1; }
tail -3 gpurun_out/p_test.log
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/p_bench.log 2>&1 && \
TMOG_XGB_PIPE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/p_bench_off.log 2>&1 && \
TMOG_PIPE_SWITCH_S=0.005 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/p_bench_g2.log 2>&1
rc=$?
for f in gpurun_out/p_bench*.log; do echo $f; python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['holdout_aupr'], d['timings'])"; done
exit $rc
