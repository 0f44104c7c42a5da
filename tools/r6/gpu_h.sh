#!/bin/bash
# round 6, call h: persistent gemm_f32m (cross-tile DMA prefetch) - tests, A/B, Householder QR
set -o pipefail
OUT=gpurun_out/r6h; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_qr.py > $OUT/test_gemm.txt 2>&1 || exit 1
echo tests ok
timeout -k 10 400 python tools/microbench/gemm_mid.py > $OUT/gemm_mid.jsonl 2>&1 || exit 2
echo bench ok
timeout -k 10 500 python tools/microbench/hh_update_ab.py blas small > $OUT/hh.jsonl 2>&1 || exit 4
echo hh ok
HEAT_GM_PERSIST=0 GM_SHAPES=upd timeout -k 10 300 python tools/microbench/gemm_mid.py > $OUT/gemm_mid_nopersist.jsonl 2>&1 || exit 5
echo ab ok
