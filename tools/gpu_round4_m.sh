#!/bin/bash
# round 4 (n): gemm_f32t accumulators started from C: GEMM/QR tests, the Householder pieces,
# the whole Householder QR, gemm 8192^3
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4n"
mkdir -p "$OUT"
cd "$ROOT"
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_gemm.py tests/test_gpu_qr.py -m gpu > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u tools/microbench/hh_parts.py > "$OUT/parts.jsonl" 2> "$OUT/parts.err" && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh.jsonl" 2> "$OUT/hh.err" && \
timeout -k 10 200 python -u tools/microbench/gemm_bench.py 8192x8192x8192 > "$OUT/gemm.txt" 2>&1
rc=$?
tail -n 3 "$OUT/tests.txt"; cat "$OUT/parts.jsonl" "$OUT/hh.jsonl"; cut -c1-400 "$OUT/gemm.txt"
echo "chain rc=$rc"
exit $rc
