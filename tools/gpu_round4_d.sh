#!/bin/bash
# round 4 (d): certified one-term kNN (h1_topk) - its GPU test, the knn tests, bench.py knn with
# and without the certified pass, kernel trace of the top-k target
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4d"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_oracle.py tests/test_gpu_select.py -m gpu -k "knn or topk or neighbor or kneigh or certified" \
  > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py --workload knn --steps 2 --warmup 1 > "$OUT/knn_h1.json" 2> "$OUT/knn_h1.err" && \
HEAT_KNN_CERTIFIED=0 timeout -k 10 300 python -u bench.py --workload knn --steps 2 --warmup 1 > "$OUT/knn_h3.json" 2> "$OUT/knn_h3.err" && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_topk" -o topk -- python3 "$ROOT/tools/microbench/pmc_targets.py" topk > "$OUT/prof_topk.log" 2>&1 )
rc=$?
find "$OUT" -name '*kernel_trace.csv' -delete 2>/dev/null
tail -5 "$OUT/tests.txt"; cut -c1-300 "$OUT/knn_h1.json" "$OUT/knn_h3.json"
find "$OUT" -name '*kernel_stats.csv' -exec sh -c 'echo {}; cut -d, -f1-4 {} | head -8' \;
echo "chain rc=$rc"
exit $rc
