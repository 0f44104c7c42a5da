#!/bin/bash
# round 4 (o): LDS-DMA vtc64 (vtc64d) + hh_step store skip: tests, pieces, whole Householder QR,
# A/B against the register-staged vtc64 (HEAT_VTC64_V1=1)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4o"
mkdir -p "$OUT"
cd "$ROOT"
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_qr.py tests/test_gpu_kernels.py -m gpu -k "qr or householder or vtc or gram or linalg" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u tools/microbench/hh_parts.py > "$OUT/parts.jsonl" 2> "$OUT/parts.err" && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh.jsonl" 2> "$OUT/hh.err" && \
HEAT_VTC64_V1=1 timeout -k 10 300 python -u tools/microbench/hh_parts.py > "$OUT/parts_v1.jsonl" 2> "$OUT/parts_v1.err"
rc=$?
tail -n 3 "$OUT/tests.txt"; cat "$OUT/parts.jsonl" "$OUT/parts_v1.jsonl"; grep householder "$OUT/hh.jsonl"; tail -3 "$OUT/parts.err"
echo "chain rc=$rc"
exit $rc
