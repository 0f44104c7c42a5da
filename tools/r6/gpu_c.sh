#!/bin/bash
# round 6, call c: triangular GEMM pairing / C-preload A/B + PMC of the triangular product
set -o pipefail
OUT=gpurun_out/r6c; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > $OUT/test_gemm.txt 2>&1 || exit 1
for pr in 0 1; do
  HEAT_GEMM_TRI_PAIRED=$pr timeout -k 10 300 python -m benchmarks.linalg.run --ops qr_r,qr --trials 3 > $OUT/linalg_pair$pr.jsonl 2>&1 || exit 2
done
for pl in 0 1; do
  HEAT_GEMM_F32_PRELOAD=$pl timeout -k 10 300 python tools/microbench/update_ab.py > $OUT/update_pre$pl.jsonl 2>&1 || exit 3
done
echo ab ok
cd /tmp
for pr in 0 1; do
HEAT_GEMM_TRI_PAIRED=$pr timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_tri_A$pr -o a -- python3 $ROOT/tools/microbench/pmc_targets.py tri > $ROOT/$OUT/pmc_tri_A$pr.log 2>&1 || exit 4
HEAT_GEMM_TRI_PAIRED=$pr timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_tri_F$pr -o f -- python3 $ROOT/tools/microbench/pmc_targets.py tri > $ROOT/$OUT/pmc_tri_F$pr.log 2>&1 || exit 5
done
echo pmc ok
