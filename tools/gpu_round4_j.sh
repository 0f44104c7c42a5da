#!/bin/bash
# round 4 (j): committed-state check + Householder QR breakdown
#  tests: certified kNN, exact k-means, threefry, knn
#  benches: knn (KH=16 per-half lists), Householder QR 1.25e6 x 4096 (time + kernel trace)
#  profiles: randn kernel trace (branch-free Kundu table lookup)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4j"
mkdir -p "$OUT"
cd "$ROOT"
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_kernels.py tests/test_gpu_oracle.py -m gpu \
  -k "certified or exact or threefry or knn" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py --workload knn --steps 2 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err" && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh.jsonl" 2> "$OUT/hh.err" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_hh" -o hh -- python3 "$ROOT/tools/microbench/hh_prof.py" 1250000 4096 > "$OUT/prof_hh.log" 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_randn" -o randn -- python3 "$ROOT/tools/microbench/pmc_targets.py" randn > "$OUT/prof_randn.log" 2>&1
rc=$?
cd "$ROOT"
find "$OUT" -name '*kernel_trace.csv' -delete 2>/dev/null
tail -n 2 "$OUT/tests.txt"; cat "$OUT/hh.jsonl"; cut -c1-300 "$OUT/knn.json"
echo "chain rc=$rc"
exit $rc
