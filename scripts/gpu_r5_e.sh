#!/bin/bash
# Exclusive (serialized) per-learner costs: one lane, one boosting part, one stream -- wall times per learner and a
# kernel trace whose durations are not inflated by concurrent streams.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
TMOG_LEARNER_LANES=1 TMOG_XGB_PIPE=1 TMOG_FIT_PHASES=1 timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --verbose > gpurun_out/r5e_serial.log 2>&1 || { tail -20 gpurun_out/r5e_serial.log; exit 1; }
grep -a '^{' gpurun_out/r5e_serial.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"fit_phases": {[^}]*}\|"timings": {[^}]*}'
D=/tmp/tr_serial
rm -rf $D
TMOG_LEARNER_LANES=1 TMOG_XGB_PIPE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/r5e_trace_run.log 2>&1 || exit $?
S=$(find $D -name '*kernel_stats.csv' | head -n 1)
T=$(find $D -name '*kernel_trace.csv' | head -n 1)
python3 scripts/kstats.py $S 2 45 > gpurun_out/r5e_serial_kstats.txt || exit $?
python3 scripts/xgb_levels.py $T --last > gpurun_out/r5e_xgb_levels.txt || exit $?
cat gpurun_out/r5e_serial_kstats.txt gpurun_out/r5e_xgb_levels.txt
