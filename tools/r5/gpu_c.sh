#!/bin/bash
# round 5 (c): small-k variants A/B (+ numerics), exact cdist epilogue, SUSY timings
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5e"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
true && \
true && \
timeout -k 10 800 python -u tools/microbench/smallk_ab.py > "$OUT/smallk_ab.jsonl" 2>&1 && \
timeout -k 10 200 python -u -m benchmarks.distance_matrix.run --case susy > "$OUT/susy.txt" 2>&1 && \
timeout -k 10 300 python -u -m benchmarks.linalg.run --ops gram > "$OUT/gram.txt" 2>&1 && \
timeout -k 10 300 python -u -m benchmarks.linalg.run --ops gram --precision high >> "$OUT/gram.txt" 2>&1 && \
HEAT_GRAM_MIN_N=100000 timeout -k 10 300 python -u -m benchmarks.linalg.run --ops gram >> "$OUT/gram.txt" 2>&1
rc=$?
cat "$OUT/smallk_ab.jsonl"; cut -c1-250 "$OUT/susy.txt" "$OUT/gram.txt"
echo "chain rc=$rc"
exit $rc
