#!/bin/bash
# round 6, call l: gemm_f32m fused split-K epilogue - tests, A/B (HEAT_GM_FUSED=0/1), bench qr
set -o pipefail
OUT=gpurun_out/r6l; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_qr.py > $OUT/test_gemm.txt 2>&1 || exit 1
echo tests ok
GM_SHAPES=sq timeout -k 10 300 python tools/microbench/gemm_mid.py > $OUT/gemm_mid_fused.jsonl 2>&1 || exit 2
HEAT_GM_FUSED=0 GM_SHAPES=sq timeout -k 10 300 python tools/microbench/gemm_mid.py > $OUT/gemm_mid_unfused.jsonl 2>&1 || exit 3
echo bench ok
timeout -k 10 300 python -u bench.py --workload qr --steps 3 --warmup 1 > $OUT/qr1.json 2> $OUT/qr1.err || exit 4
echo qr ok
