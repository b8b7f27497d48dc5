#!/bin/bash
# Concurrent learner lanes: GPU equality test, then the headline with lanes on / off on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-lanes}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_concurrent_lanes.py tests/test_tree_engine.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_test.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --verbose > gpurun_out/${T}_on.log 2>&1 && \
TMOG_LEARNER_LANES=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --verbose > gpurun_out/${T}_off.log 2>&1
rc=$?
tail -n 3 gpurun_out/${T}_test.log; for f in on off; do grep '^{' gpurun_out/${T}_$f.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['holdout_aupr'], d['best_model'], d['timings'])"; done
exit $rc
