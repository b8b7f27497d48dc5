#!/bin/bash
# Generic on/off A/B of an env switch on the headline (same box, interleaved), after the tree / learner GPU tests,
# plus a kernel-stats profile of the default: bash scripts/gpu_s3_ab.sh TAG VAR
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-ab}; V=${2:-X}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py tests/test_gpu_kernels.py tests/test_forest_share.py tests/test_tree_capacity.py tests/test_learner_parallel.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_test.log 2>&1 || { tail -n 30 gpurun_out/${T}_test.log; exit 1; }
tail -n 1 gpurun_out/${T}_test.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --verbose > gpurun_out/${T}_${tag}.log 2>&1 || return $?
  grep '^{' gpurun_out/${T}_${tag}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$tag', round(d['value'],4), d['holdout_aupr'], {k: round(v,3) for k,v in d['timings'].items()})"
}
run on X=1 && run off $V=0 && run on2 X=1 && run off2 $V=0 || exit $?
D=/tmp/prof_$T; rm -rf $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/${T}_prof.log 2>&1 || exit $?
cp $D/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv && python3 scripts/kstats.py gpurun_out/${T}_kernel_stats.csv > gpurun_out/${T}_kstats.txt; head -12 gpurun_out/${T}_kstats.txt
