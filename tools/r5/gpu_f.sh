#!/bin/bash
# round 5 (f): 4x4x1 MFMA layout probe; 128-tile split-K GEMM tests + A/B vs hipBLASLt; QR with the
# native rank update
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5f"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probes/mfma4x4_probe > "$OUT/probe.txt" 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests_gemm.txt" 2>&1 && \
timeout -k 10 400 python -u tools/microbench/gemm_small.py > "$OUT/gemm_small.jsonl" 2>&1 && \
timeout -k 10 300 python -u -m benchmarks.linalg.run --ops matmul,qr > "$OUT/linalg_blas.txt" 2>&1 && \
HEAT_HH_UPDATE=small timeout -k 10 300 python -u -m benchmarks.linalg.run --ops qr > "$OUT/linalg_small.txt" 2>&1
rc=$?
tail -n 2 "$OUT/tests_gemm.txt"; cat "$OUT/gemm_small.jsonl"; cut -c1-250 "$OUT/linalg_blas.txt" "$OUT/linalg_small.txt"
echo "chain rc=$rc"
exit $rc
