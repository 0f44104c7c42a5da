#!/bin/bash
# round 4 (w): full GPU test suite, smoke, default bench, knn bench
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4w"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err"
rc=$?
tail -n 3 "$OUT/tests.txt"; tail -1 "$OUT/smoke.txt"; cat "$OUT/bench.json" "$OUT/knn.json"
echo "chain rc=$rc"
exit $rc
