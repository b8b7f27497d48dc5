#!/bin/bash
# Tree-kernel change check: tree GPU identity tests, headline bench (10 steps), kernel stats of one step.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-hist}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_tree_engine.py tests/test_gpu_kernels.py tests/test_forest_share.py tests/test_tree_capacity.py tests/test_mlp.py tests/test_sparse_linear_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_test.log 2>&1
rc=$?; tail -n 2 gpurun_out/${T}_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --verbose > gpurun_out/${T}_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/${T}_bench.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('bench', round(d['value'],4), d['holdout_aupr'], {k: round(v,3) for k,v in d['timings'].items()})"
D=/tmp/prof_$T; rm -rf $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/${T}_prof.log 2>&1 || exit $?
cp $D/run_kernel_stats.csv gpurun_out/${T}_kernel_stats.csv && python3 scripts/kstats.py gpurun_out/${T}_kernel_stats.csv > gpurun_out/${T}_kstats.txt; head -12 gpurun_out/${T}_kstats.txt
