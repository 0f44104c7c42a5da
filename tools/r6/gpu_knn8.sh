#!/bin/bash
# round 6: PMC rows of the kNN screening kernel, round-5 form (HEAT_H1_CFG=o) vs the 8-wave default,
# shipped and without refill DMA (HEAT_H1_DEBUG=4, invalid results by design)
set -o pipefail
OUT=gpurun_out/r6knn8; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
cd /tmp
for v in o:0 g:0 g:4 o:4; do
  c=${v%%:*}; d=${v##*:}
  HEAT_H1_CFG=$c HEAT_H1_DEBUG=$d timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_${c}$d -o a -- python3 $ROOT/tools/microbench/pmc_targets.py knn > $ROOT/$OUT/pmc_${c}$d.log 2>&1 || exit 1
  echo "$c$d ok"
done
for c in o g; do
  HEAT_H1_CFG=$c timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_l$c -o l -- python3 $ROOT/tools/microbench/pmc_targets.py knn > $ROOT/$OUT/pmc_l$c.log 2>&1 || exit 2
  echo "l$c ok"
done
