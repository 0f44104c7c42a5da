#!/bin/bash
# round 6: where the kNN screening kernel's time goes - one PMC pass (SQ issue / MFMA counters) per
# HEAT_H1_DEBUG variant (results invalid by design in the variants: 1 no selection, 2 no chunk
# barrier, 4 no refill DMA (the ring keeps its first chunks), 7 all three off)
set -o pipefail
OUT=gpurun_out/r6knnd; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
cd /tmp
for d in 0 1 2 4 7; do
  HEAT_H1_DEBUG=$d timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_d$d -o a -- python3 $ROOT/tools/microbench/pmc_targets.py knn > $ROOT/$OUT/pmc_d$d.log 2>&1 || exit 1
  echo "d$d ok"
done
for d in 0 7; do
  HEAT_H1_DEBUG=$d timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_l$d -o l -- python3 $ROOT/tools/microbench/pmc_targets.py knn > $ROOT/$OUT/pmc_l$d.log 2>&1 || exit 2
  echo "l$d ok"
done
