#!/bin/bash
# round 6: clock / MFMA-busy / traffic of hipBLASLt vs gemm_f32m at 6144^3 (one PMC pass per group)
set -o pipefail
OUT=gpurun_out/r6w; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $ROOT/$OUT/pa -o a -- python3 $ROOT/tools/microbench/pmc_targets.py libvsmid > $ROOT/$OUT/pa.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $ROOT/$OUT/pf -o f -- python3 $ROOT/tools/microbench/pmc_targets.py libvsmid > $ROOT/$OUT/pf.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $ROOT/$OUT/pw -o w -- python3 $ROOT/tools/microbench/pmc_targets.py libvsmid > $ROOT/$OUT/pw.log 2>&1 || exit 3
echo ok
