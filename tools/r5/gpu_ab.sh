#!/bin/bash
# round 5 (ab): fused small-k Lloyd epilogue: numerics, per-step times, reference protocol, bench
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5ab"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "kmeans or lloyd or small" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/smallk_fitloop2.py > "$OUT/fitloop.jsonl" 2> "$OUT/fitloop.err" && \
timeout -k 10 300 python -u -m benchmarks.kmeans.run --case reference --trials 5 > "$OUT/ref.jsonl" 2> "$OUT/ref.err" && \
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
tail -n 1 "$OUT/tests.txt"; cut -c1-200 "$OUT/fitloop.jsonl"; grep median "$OUT/ref.jsonl" | cut -c1-400; cut -c1-200 "$OUT/bench.json"
echo "chain rc=$rc"
exit $rc
