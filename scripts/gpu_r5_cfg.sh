#!/bin/bash
# The secondary BASELINE configs (3 timed steps each) + a kernel-stats trace of multiclass-text.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in multiclass-text lr-rf-1m regression-100m; do
  timeout -k 10 600 python3 -u bench.py --config $cfg --steps 3 --warmup 1 --verbose > gpurun_out/r5cfg_$cfg.log 2>&1 || { tail -20 gpurun_out/r5cfg_$cfg.log; exit 1; }
  echo "$cfg $(grep -a '^{' gpurun_out/r5cfg_$cfg.log | grep -o '"value": [0-9.]*\|"holdout_[a-z]*": [0-9.e-]*' | tr '\n' ' ')"
  grep -a '^{' gpurun_out/r5cfg_$cfg.log | grep -o '"timings": {[^}]*}\|"top_stages": {[^}]*}'
done
D=/tmp/tr_mct
rm -rf $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --config multiclass-text --steps 1 --warmup 1 > gpurun_out/r5cfg_mct_trace.log 2>&1 || exit $?
S=$(find $D -name '*kernel_stats.csv' | head -n 1)
python3 scripts/kstats.py $S 2 30 > gpurun_out/r5cfg_mct_kstats.txt || exit $?
head -32 gpurun_out/r5cfg_mct_kstats.txt
