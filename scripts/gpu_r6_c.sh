#!/bin/bash
# Round 6 projections (one GPU, parallel/dist.py simulate): default schedule at world 2 and 4 (every rank), forced
# hybrid groups (feature-parallel XGBoost on the device-planned loop, exchange answered locally) at world 4 and 8.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 400 python3 -u scripts/project_schedule.py --world 2 --out $O/proj2 > $O/proj2.out 2>&1 || { tail -20 $O/proj2.out; exit 1; }
tail -1 $O/proj2.out
timeout -k 10 500 python3 -u scripts/project_schedule.py --world 4 --out $O/proj4 > $O/proj4.out 2>&1 || { tail -20 $O/proj4.out; exit 1; }
tail -1 $O/proj4.out
TMOG_PARALLEL_MODE=hybrid:2 timeout -k 10 300 python3 -u scripts/project_schedule.py --world 4 --ranks 0,2 --out $O/proj4h2 > $O/proj4h2.out 2>&1 || { tail -20 $O/proj4h2.out; exit 1; }
tail -1 $O/proj4h2.out
