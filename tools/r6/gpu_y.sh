#!/bin/bash
# round 6: the paired-barrier gemm_f32m form in the plan - GEMM / QR GPU tests, square microbench
set -o pipefail
OUT=gpurun_out/r6y; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_qr.py > $OUT/tests.txt 2>&1 || exit 1
GM_SHAPES=sq timeout -k 10 400 python -u tools/microbench/gemm_mid.py > $OUT/gemm_mid.jsonl 2> $OUT/gemm_mid.err || exit 2
echo ok
