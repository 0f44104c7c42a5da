#!/bin/bash
# h3_cscale grid-stride rewrite: k-means / KNN / certified-filter GPU tests, the oracle checks,
# the flagship bench, then a kernel-trace of the top-k target (h3_cscale time)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_oracle.py -m gpu -k "knn or kmeans or h3 or certified or assign or oracle or topk" \
  > "$OUT/t_cscale.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py > "$OUT/bench_cscale.json" 2> "$OUT/bench_cscale.err" && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_topk2" -o topk -- python3 "$ROOT/tools/microbench/pmc_targets.py" topk > "$OUT/prof_topk2.log" 2>&1 )
rc=$?
find "$OUT/prof_topk2" -name '*kernel_trace.csv' -delete 2>/dev/null
tail -3 "$OUT/t_cscale.txt"; cut -c1-200 "$OUT/bench_cscale.json"
echo "chain rc=$rc"
exit $rc
