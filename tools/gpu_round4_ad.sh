#!/bin/bash
# round 4 (ad): end-of-round check: full GPU test suite, smoke, default bench, knn + cdist benches,
# kernel trace of the default bench
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4ad"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/tests.txt" 2>&1; \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bench" -o bench -- python3 -u bench.py --steps 10 --warmup 3 --exact-steps 0 > "$OUT/prof_bench.log" 2>&1
rc=$?
tail -n 2 "$OUT/tests.txt"; tail -1 "$OUT/smoke.txt"; cat "$OUT/bench.json" "$OUT/knn.json" | cut -c1-400
echo "chain rc=$rc"
exit $rc
