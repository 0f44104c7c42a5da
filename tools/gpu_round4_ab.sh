#!/bin/bash
# round 4 (ab): framework overhead after the where / index-shape fixes, small-GEMM sweep, GPU
# parity + core tests
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4ab"
mkdir -p "$OUT"
cd "$ROOT"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_parity.py tests/test_gpu_framework.py tests/test_gpu_select.py tests/test_gpu_gemm.py tests/test_gpu_qr.py -m gpu > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/ops_overhead.py > "$OUT/ops.jsonl" 2> "$OUT/ops.err" && \
timeout -k 10 300 python -u tools/microbench/gemm_small.py > "$OUT/gemm_small.jsonl" 2> "$OUT/gemm_small.err"
rc=$?
tail -n 2 "$OUT/tests.txt"; cat "$OUT/ops.jsonl" "$OUT/gemm_small.jsonl"; tail -2 "$OUT/gemm_small.err"
echo "chain rc=$rc"
exit $rc
