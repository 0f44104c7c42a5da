#!/bin/bash
# round 5 (t): 128-tile GEMM with pipelined fragment reads + unguarded interior loads: numerics,
# the small-GEMM table, the Householder update A/B (library vs 128-tile)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5t"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u tools/microbench/gemm_small.py > "$OUT/gemm_small.jsonl" 2> "$OUT/gemm_small.err" && \
timeout -k 10 600 python -u tools/microbench/hh_update_ab.py blas small > "$OUT/hh_ab.jsonl" 2> "$OUT/hh_ab.err"
rc=$?
tail -n 2 "$OUT/tests.txt"; cat "$OUT/gemm_small.jsonl" | cut -c1-300; cat "$OUT/hh_ab.jsonl"
echo "chain rc=$rc"
exit $rc
