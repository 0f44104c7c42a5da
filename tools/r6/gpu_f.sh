#!/bin/bash
# round 6, call f: gemm_f32m with the 32-bit-offset epilogue - tests, NBUF 4 / 3 A/B, Householder QR
# with the native (gemm_f32m) trailing update
set -o pipefail
OUT=gpurun_out/r6f; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "small_layouts or mid_update" > $OUT/test_gemm.txt 2>&1 || exit 1
echo tests ok
timeout -k 10 400 python tools/microbench/gemm_mid.py > $OUT/gemm_mid4.jsonl 2>&1 || exit 2
HEAT_GM_NBUF=3 timeout -k 10 400 python tools/microbench/gemm_mid.py > $OUT/gemm_mid3.jsonl 2>&1 || exit 3
echo bench ok
timeout -k 10 500 python tools/microbench/hh_update_ab.py blas small > $OUT/hh4.jsonl 2>&1 || exit 4
HEAT_GM_NBUF=3 timeout -k 10 300 python tools/microbench/hh_update_ab.py small > $OUT/hh3.jsonl 2>&1 || exit 4
echo hh ok
