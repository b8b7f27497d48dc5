#!/bin/bash
# 8- vs 4-wave histogram workgroups: tree GPU tests, then the headline A/B (TMOG_HIST_WAVES) and a kernel-stats
# profile of the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-w}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py tests/test_gpu_kernels.py tests/test_forest_share.py tests/test_tree_capacity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_test.log 2>&1 || { tail -n 20 gpurun_out/${T}_test.log; exit 1; }
tail -n 1 gpurun_out/${T}_test.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --verbose > gpurun_out/${T}_${tag}.log 2>&1 || return $?
  grep '^{' gpurun_out/${T}_${tag}.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$tag', round(d['value'],4), d['holdout_aupr'], {k: round(v,3) for k,v in d['timings'].items()})"
}
run w8 X=1 && run w4 TMOG_HIST_WAVES=4 && run w8b X=1 && run w4b TMOG_HIST_WAVES=4 || exit $?
D=/tmp/prof_$T; rm -rf $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/${T}_prof.log 2>&1 || exit $?
cp $D/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv && python3 scripts/kstats.py gpurun_out/${T}_kernel_stats.csv > gpurun_out/${T}_kstats.txt; head -8 gpurun_out/${T}_kstats.txt
