#!/bin/bash
# round 4 (k): Householder QR pieces (panel strided vs compact, K=256 update gemm_f32t vs
# hipBLASLt, vtc64) and the two-level outer width 512 vs 256
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4k"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u tools/microbench/hh_parts.py > "$OUT/parts.jsonl" 2> "$OUT/parts.err" && \
HEAT_HH_OUTER=512 timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh512.jsonl" 2> "$OUT/hh512.err"
rc=$?
cat "$OUT/parts.jsonl" "$OUT/hh512.jsonl"; tail -3 "$OUT/parts.err"
echo "chain rc=$rc"
exit $rc
