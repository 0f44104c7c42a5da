#!/bin/bash
# round 6, call e: LDS-DMA 128-tile GEMM (gemm_f32m) - tests, A/B vs gemm_f32s / hipBLASLt, PMC
set -o pipefail
OUT=gpurun_out/r6e; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "small_layouts or mid_update" > $OUT/test_gemm.txt 2>&1 || exit 1
echo tests ok
timeout -k 10 400 python tools/microbench/gemm_mid.py > $OUT/gemm_mid.jsonl 2>&1 || exit 2
HEAT_GM_NBUF=3 GM_SHAPES=upd timeout -k 10 300 python tools/microbench/gemm_mid.py > $OUT/gemm_mid_nbuf3.jsonl 2>&1 || exit 3
echo bench ok
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_mid_A -o a -- python3 $ROOT/tools/microbench/pmc_targets.py mid > $ROOT/$OUT/pmc_mid_A.log 2>&1 || exit 5
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_mid_F -o f -- python3 $ROOT/tools/microbench/pmc_targets.py mid > $ROOT/$OUT/pmc_mid_F.log 2>&1 || exit 6
echo pmc ok
