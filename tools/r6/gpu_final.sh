#!/bin/bash
# round 6: full GPU test suite, smoke, default bench, kNN and QR benches
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/${R6FINAL_DIR:-r6final}"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 960 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > "$OUT/tests.txt" 2>&1
trc=$?
echo "tests rc=$trc" >> "$OUT/tests.txt"
if [ $trc -eq 0 ] || [ $trc -eq 1 ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 && \
  timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
  timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err" && \
  timeout -k 10 300 python -u bench.py --workload qr --steps 3 --warmup 1 > "$OUT/qr.json" 2> "$OUT/qr.err"
  rc=$?
else
  rc=$trc
fi
tail -n 15 "$OUT/tests.txt"; tail -1 "$OUT/smoke.txt"; cut -c1-300 "$OUT/bench.json" "$OUT/knn.json" "$OUT/qr.json"
echo "chain rc=$rc"
exit $rc
