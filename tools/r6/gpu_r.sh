#!/bin/bash
# round 6, call r: vectorised fp64 slice sums (Gram) - QR
# tests, TSQR benchmark, kernel trace of the factor
set -o pipefail
OUT=gpurun_out/r6s; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qr.py tests/test_gpu_gemm.py -k "gram or qr or cholesky or householder or tri or split" > $OUT/test_qr.txt 2>&1 || exit 1
echo tests ok
timeout -k 10 400 python -m benchmarks.linalg.run --ops gram,qr_r,qr --trials 3 > $OUT/linalg.jsonl 2>&1 || exit 2
echo bench ok
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/qrtrace -o qr -- python3 -m benchmarks.linalg.run --ops qr --trials 1 > $ROOT/$OUT/qrtrace.log 2>&1 || exit 3
echo trace ok
