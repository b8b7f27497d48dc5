#!/bin/bash
# Diagnostic: time of the histogram kernel by item kind (CSR / dense) on the XGBoost phase.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hs
export TMPDIR=/tmp
for D in 0 1 2; do
  TMOG_HIST_DEBUG=$D timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/hs/d$D -o s -- python3 bench.py --rows 2000000 --steps 1 --warmup 0 --models OpXGBoostClassifier > gpurun_out/hs/d$D.log 2>&1 || exit 1
done
find gpurun_out -name '*trace*.csv' -delete; find gpurun_out -name '*.db' -delete
for D in 0 1 2; do grep -h "hist_build_kernel<2>\|split_scan_kernel<2>" gpurun_out/hs/d$D/s_kernel_stats.csv | cut -d, -f1-3 | cut -c1-40,150-; done
