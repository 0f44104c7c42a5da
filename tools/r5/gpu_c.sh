#!/bin/bash
# round 5 (c): small-k variants A/B (+ numerics), exact cdist epilogue, SUSY timings
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5c"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "small or cdist" > "$OUT/tests.txt" 2>&1 && \
HEAT_KS_VARIANT=wave timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "kmeans_step_small or small_k" > "$OUT/tests_wave.txt" 2>&1 && \
timeout -k 10 400 python -u tools/microbench/smallk_ab.py > "$OUT/smallk_ab.jsonl" 2>&1 && \
timeout -k 10 200 python -u -m benchmarks.distance_matrix.run --case susy > "$OUT/susy.txt" 2>&1
rc=$?
tail -n 2 "$OUT/tests.txt" "$OUT/tests_wave.txt"; cat "$OUT/smallk_ab.jsonl"; cut -c1-250 "$OUT/susy.txt"
echo "chain rc=$rc"
exit $rc
