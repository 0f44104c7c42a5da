#!/bin/bash
# round 6, call n: the plan with the 64 x 64 tile - GEMM/QR tests, the square shapes through fgemm
set -o pipefail
OUT=gpurun_out/r6n; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_qr.py > $OUT/test_gemm.txt 2>&1 || exit 1
echo tests ok
GM_SHAPES=sq timeout -k 10 300 python tools/microbench/gemm_mid.py > $OUT/gemm_mid.jsonl 2>&1 || exit 2
echo bench ok
HEAT_GM64_MAXK=64 timeout -k 10 300 python tools/microbench/hh_update_ab.py small > $OUT/hh_k64.jsonl 2>&1 || exit 3
timeout -k 10 300 python tools/microbench/hh_update_ab.py small > $OUT/hh_k0.jsonl 2>&1 || exit 4
echo hh ok
