#!/bin/bash
# round 5 (u): the kNN kernel as committed (queue Q = 4, half-wave rank-1 DMA pieces) and the
# pipelined 128-tile GEMM: numerics, kNN A/B + bench, small-GEMM table, Householder update A/B
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5u"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "knn or topk or gemm or matmul or gram" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/h1_ab.py 0 1 3 > "$OUT/h1_ab.jsonl" 2> "$OUT/h1_ab.err" && \
HEAT_H1_CFG=w8 timeout -k 10 100 python -u tools/microbench/h1_ab.py 0 >> "$OUT/h1_ab.jsonl" 2>> "$OUT/h1_ab.err" && \
timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err" && \
timeout -k 10 300 python -u tools/microbench/gemm_small.py > "$OUT/gemm_small.jsonl" 2> "$OUT/gemm_small.err" && \
timeout -k 10 600 python -u tools/microbench/hh_update_ab.py blas small > "$OUT/hh_ab.jsonl" 2> "$OUT/hh_ab.err"
rc=$?
tail -n 2 "$OUT/tests.txt"; cat "$OUT/h1_ab.jsonl"; cut -c1-400 "$OUT/knn.json"; cut -c1-300 "$OUT/gemm_small.jsonl"; cat "$OUT/hh_ab.jsonl"
echo "chain rc=$rc"
exit $rc
