#!/bin/bash
# round 5 (a): small-k kernel rewrite check + timing, default bench, 2-GPU-free contract
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5a"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "small" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/smallk_bench.py > "$OUT/smallk.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" && \
timeout -k 10 200 python -u -m benchmarks.kmeans.run --case reference > "$OUT/kref.txt" 2>&1
rc=$?
tail -n 3 "$OUT/tests.txt"; cat "$OUT/smallk.txt"; cut -c1-300 "$OUT/bench.json"; tail -5 "$OUT/kref.txt"
echo "chain rc=$rc"
exit $rc
