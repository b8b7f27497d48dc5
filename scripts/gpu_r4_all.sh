#!/bin/bash
# The secondary BASELINE configs on 1 MI355X (verbose stage timings), one box, plus regression-100m with a 20M-row
# training sample (tree learners above 2^24 training rows).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r4all}
timeout -k 10 500 python -u bench.py --config regression-100m --steps 2 --warmup 1 --verbose > gpurun_out/${T}_reg.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config multiclass-text --steps 3 --warmup 1 --verbose > gpurun_out/${T}_mct.log 2>&1 && \
timeout -k 10 400 python -u bench.py --config lr-rf-1m --steps 3 --warmup 1 --verbose > gpurun_out/${T}_lrrf.log 2>&1 && \
timeout -k 10 900 python -u bench.py --config regression-100m --max-training-sample 20000000 --steps 1 --warmup 1 --verbose > gpurun_out/${T}_reg20m.log 2>&1
rc=$?
for f in gpurun_out/${T}_*.log; do echo "== $f"; grep -a '^{' $f | grep -o '"value": [0-9.]*\|"holdout_[a-z]*": [0-9.e-]*\|"timings": {[^}]*}\|"peak_hbm_gb_per_gpu": [0-9.]*'; done
exit $rc
