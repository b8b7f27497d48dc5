#!/bin/bash
# single-workgroup planner / finaliser at 256 threads: resident-grower tests under it, then a headline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TMOG_PLAN_THREADS=256 timeout -k 10 400 python3 -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_tree_resident_gpu.py tests/test_native_alloc_gpu.py tests/test_gpu_kernels.py > gpurun_out/r5_pt_tests.log 2>&1 || { tail -30 gpurun_out/r5_pt_tests.log; exit 1; }
tail -1 gpurun_out/r5_pt_tests.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --verbose > gpurun_out/r5pt_$tag.log 2>&1 || { tail -20 gpurun_out/r5pt_$tag.log; return 1; }
  echo "$tag $(grep -a '^{' gpurun_out/r5pt_$tag.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"OpXGBoostClassifier": [0-9.]*' | tr '\n' ' ')"
}
run base || exit 1
run t256 TMOG_PLAN_THREADS=256 || exit 1
run t256nolds TMOG_PLAN_THREADS=256 TMOG_PLAN_LDS=0 || exit 1
run t512 TMOG_PLAN_THREADS=512 || exit 1
run base2 || exit 1
run t256b TMOG_PLAN_THREADS=256 || exit 1
