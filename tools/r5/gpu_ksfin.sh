#!/bin/bash
# small-k Lloyd step with the w2 pass: epilogue as reduction + one-block finish (default) vs fused
# last-block form (HEAT_KS_FIN=fused); numerics, fit loop, reference protocol, default bench
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT" TMPDIR=/tmp
OUT="$ROOT/gpurun_out/r5ksfin"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "kmeans or lloyd or small" > "$OUT/tests.txt" 2>&1 || exit $?
for v in split fused split fused; do
  HEAT_KS_FIN=$v timeout -k 10 200 python -u tools/microbench/smallk_fitloop2.py > "$OUT/fit_$v.jsonl" 2>&1 || exit $?
  HEAT_KS_FIN=$v timeout -k 10 300 python -u -m benchmarks.kmeans.run --case reference --trials 5 >> "$OUT/ref_$v.jsonl" 2>> "$OUT/ref.err" || exit $?
  echo "$v $(grep -o '"mean": [0-9.]*' $OUT/fit_$v.jsonl | head -1) ref $(grep -o '"median_s": [0-9.]*' $OUT/ref_$v.jsonl | tail -1)"
done
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
tail -n 1 "$OUT/tests.txt"; cut -c1-200 "$OUT/bench.json"
