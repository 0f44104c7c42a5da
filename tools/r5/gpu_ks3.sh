#!/bin/bash
# small-k: tail folded into the w2 pass + unrolled partial reduction; numerics, fit loop, reference protocol, trace
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT" TMPDIR=/tmp
OUT="$ROOT/gpurun_out/r5ks3"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "kmeans or lloyd or small or KMeans" > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -n 1 "$OUT/tests.txt"
for i in 1 2; do
  timeout -k 10 200 python -u tools/microbench/smallk_fitloop2.py > "$OUT/fit_$i.jsonl" 2>&1 || exit $?
  timeout -k 10 300 python -u -m benchmarks.kmeans.run --case reference --trials 5 >> "$OUT/ref.jsonl" 2>> "$OUT/ref.err" || exit $?
  echo "$(grep -o '^{"[a-z_A-Z0-9]*"\|"mean": [0-9.]*' $OUT/fit_$i.jsonl | paste - - | tr '\n' ' ') ref $(grep -o '"median_s": [0-9.]*' $OUT/ref.jsonl | tail -1)"
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o t -- python3 "$ROOT/tools/microbench/smallk_trace.py" > "$OUT/tr.log" 2>&1
