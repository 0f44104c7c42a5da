#!/bin/bash
# round 4 (ac): library dispatch for GEMMs with few output tiles: linalg / gemm / dist tests,
# framework overhead, linalg bench at the north-star shape
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4ac"
mkdir -p "$OUT"
cd "$ROOT"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $T tests/test_gpu_gemm.py tests/test_gpu_qr.py tests/test_gpu_parity.py tests/test_gpu_framework.py tests/test_gpu_dist.py -m gpu > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/ops_overhead.py > "$OUT/ops.jsonl" 2> "$OUT/ops.err" && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py > "$OUT/linalg.jsonl" 2> "$OUT/linalg.err"
rc=$?
tail -n 2 "$OUT/tests.txt"; grep matmul "$OUT/ops.jsonl"; cat "$OUT/linalg.jsonl"
echo "chain rc=$rc"
exit $rc
