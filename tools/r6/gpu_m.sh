#!/bin/bash
# round 6, call m: gemm_f32m wait-count fix (256 x 128 re-measured) + 64 x 64 tiles - tests, A/B, Householder QR, PMC
set -o pipefail
OUT=gpurun_out/r6m; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_qr.py > $OUT/test_gemm.txt 2>&1 || exit 1
echo tests ok
timeout -k 10 400 python tools/microbench/gemm_mid.py > $OUT/gemm_mid.jsonl 2>&1 || exit 2
echo bench ok
HEAT_GM_WIDE=1 timeout -k 10 500 python tools/microbench/hh_update_ab.py small > $OUT/hh_wide.jsonl 2>&1 || exit 4
echo hh ok
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_mid_A -o a -- python3 $ROOT/tools/microbench/pmc_targets.py mid > $ROOT/$OUT/pmc_mid_A.log 2>&1 || exit 5
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_mid_F -o f -- python3 $ROOT/tools/microbench/pmc_targets.py mid > $ROOT/$OUT/pmc_mid_F.log 2>&1 || exit 6
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_mid_W -o w -- python3 $ROOT/tools/microbench/pmc_targets.py mid > $ROOT/$OUT/pmc_mid_W.log 2>&1 || exit 7
echo pmc ok
