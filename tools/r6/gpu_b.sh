#!/bin/bash
# round 6, call b: triangular-aware CholeskyQR2 products - tests, A/B timing, kernel trace
set -o pipefail
mkdir -p gpurun_out/r6b
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "b_upper" > gpurun_out/r6b/test_tri.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_qr.py > gpurun_out/r6b/test_qr.txt 2>&1 || exit 2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ipc.py > gpurun_out/r6b/test_ipc.txt 2>&1 || exit 6
echo tests ok
for tri in 0 1; do
  HEAT_QR_TRI=$tri timeout -k 10 300 python -m benchmarks.linalg.run --ops qr_r,qr --trials 3 > gpurun_out/r6b/linalg_tri$tri.jsonl 2>&1 || exit 3
  HEAT_QR_TRI=$tri timeout -k 10 300 python -m benchmarks.linalg.run --ops qr_r,qr --trials 3 --precision high > gpurun_out/r6b/linalg_high_tri$tri.jsonl 2>&1 || exit 4
done
echo bench ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b/prof -o tri -- python -m benchmarks.linalg.run --ops qr --trials 1 > gpurun_out/r6b/prof.log 2>&1 || exit 5
echo prof ok
