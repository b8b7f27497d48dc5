#!/bin/bash
# Round 6, first call: GPU suite + smoke at HEAD, the fp32 headline (5 steps), the XGBoost-only selector (the
# FeatureEngineering swing case), kernel statistics of the headline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6a
export TMPDIR=/tmp
O=gpurun_out/r6a
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 --verbose > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep -a '^{' $O/bench.log | grep -o '"value": [0-9.]*\|"holdout_aupr": [0-9.]*\|"dtype": "[a-z0-9]*"\|"FeatureEngineering": [0-9.]*\|"step_s": [^]]*'
timeout -k 10 400 python3 -u bench.py --models OpXGBoostClassifier --steps 3 --warmup 1 --verbose > $O/xgb_alone.log 2>&1 || { tail -20 $O/xgb_alone.log; exit 1; }
grep -a '^{' $O/xgb_alone.log | grep -o '"value": [0-9.]*\|"FeatureEngineering": [0-9.]*\|"step_s": [^]]*'
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fp -o fp -- python3 -u bench.py --steps 2 --warmup 1 > $O/prof_run.log 2>&1 || { tail -20 $O/prof_run.log; exit 1; }
F=$(find /tmp/fp -name '*kernel_stats.csv' | head -n 1)
python3 -c "
import csv
rows = list(csv.DictReader(open('$F')))
tot = sum(float(r['TotalDurationNs']) for r in rows) / 3e6
print(f'total kernel time {tot:.1f} ms per train (3 trains: 1 warm-up + 2 timed; concurrent lanes, durations include sharing)')
for r in rows[:30]: print(f\"{float(r['TotalDurationNs'])/3e6:9.1f} ms/train {int(r['Calls'])//3:6d} calls/train {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}\")
" > $O/kernel_stats.txt
head -14 $O/kernel_stats.txt
rm -rf /tmp/fp
