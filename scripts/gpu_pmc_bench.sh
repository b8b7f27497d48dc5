#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) over the XGBoost + LR phases of a reduced bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--rows ${ROWS:-2000000} --steps 1 --warmup 0 --models ${MODELS:-OpXGBoostClassifier,OpLogisticRegression}"
RX=${RX:-'hist_build|split_scan|pair_scan|partition_fused|lr_objective|level_plan|boost_epilogue|forest_predict'}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/stats -o s -- python3 bench.py $ARGS > gpurun_out/pmc/stats.log 2>&1 || exit 1
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
         "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE" "TCC_MISS_sum WRITE_SIZE" "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc/p$i -o p -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; break; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt
find gpurun_out -size +2M -delete
find gpurun_out -name '*.db' -delete
cat gpurun_out/pmc/summary.txt
