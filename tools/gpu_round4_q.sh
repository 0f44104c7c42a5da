#!/bin/bash
# round 4 (q): precision of the Householder update pieces under float32 matmul precision highest/high
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4q"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u tools/microbench/hh_prec.py > "$OUT/prec.jsonl" 2> "$OUT/prec.err"
rc=$?
cat "$OUT/prec.jsonl"; tail -3 "$OUT/prec.err"
echo "chain rc=$rc"
exit $rc
