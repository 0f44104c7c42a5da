#!/bin/bash
# round 5 (g): 128-tile GEMM + small-k 4x4x1 update + symmetric exact cdist: tests, A/B, timings
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5g"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_kernels.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "gemm or small or cdist or gram" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/smallk_bench.py > "$OUT/smallk.txt" 2>&1 && \
timeout -k 10 200 python -u -m benchmarks.distance_matrix.run --case susy > "$OUT/susy.txt" 2>&1 && \
timeout -k 10 400 python -u tools/microbench/gemm_small.py > "$OUT/gemm_small.jsonl" 2>&1 && \
timeout -k 10 300 python -u -m benchmarks.kmeans.run --case reference > "$OUT/kref.txt" 2>&1 && \
timeout -k 10 300 python -u -m benchmarks.linalg.run --ops matmul,qr > "$OUT/linalg_blas.txt" 2>&1 && \
HEAT_HH_UPDATE=small timeout -k 10 300 python -u -m benchmarks.linalg.run --ops qr > "$OUT/linalg_small.txt" 2>&1
rc=$?
tail -n 3 "$OUT/tests.txt"; cat "$OUT/smallk.txt"; cut -c1-260 "$OUT/susy.txt" "$OUT/kref.txt"; cat "$OUT/gemm_small.jsonl"; cut -c1-250 "$OUT/linalg_blas.txt" "$OUT/linalg_small.txt"
echo "chain rc=$rc"
exit $rc
