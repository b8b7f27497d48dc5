#!/bin/bash
# Round 6 projections at world 8: the default schedule (every rank) and hybrid groups of 4 (one rank per group).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6d
mkdir -p $O
TMOG_PARALLEL_MODE=hybrid:4 timeout -k 10 300 python3 -u scripts/project_schedule.py --world 8 --ranks 0,4 --out $O/proj8h4 > $O/proj8h4.out 2>&1 || { tail -20 $O/proj8h4.out; exit 1; }
tail -1 $O/proj8h4.out
timeout -k 10 800 python3 -u scripts/project_schedule.py --world 8 --out $O/proj8 > $O/proj8.out 2>&1 || { tail -20 $O/proj8.out; exit 1; }
tail -1 $O/proj8.out
