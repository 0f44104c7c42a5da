#!/bin/bash
# round 4 (t): Householder accuracy per V^T C variant vs LAPACK-style fp32 QR; pieces; whole QR
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4t"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 500 python -u tools/microbench/hh_variants.py > "$OUT/var.jsonl" 2> "$OUT/var.err" && \
timeout -k 10 300 python -u tools/microbench/hh_parts.py > "$OUT/parts.jsonl" 2> "$OUT/parts.err" && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh.jsonl" 2> "$OUT/hh.err" && \
HEAT_VTC_KCHUNK=1024 timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh1024.jsonl" 2> "$OUT/hh1024.err"
rc=$?
cat "$OUT/var.jsonl" "$OUT/parts.jsonl"; grep householder "$OUT/hh.jsonl" "$OUT/hh1024.jsonl"; tail -3 "$OUT/var.err"
echo "chain rc=$rc"
exit $rc
