#!/bin/bash
# round 4 (v): fused kNN rescoring kernel + 32-candidate certified lists: tests, bench knn A/B
# (HEAT_KNN_KP=16 vs 32), kernel trace of the 32 form
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4v"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_kernels.py -m gpu -k "knn or topk" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > "$OUT/knn32.json" 2> "$OUT/knn32.err" && \
HEAT_KNN_KP=16 timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > "$OUT/knn16.json" 2> "$OUT/knn16.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o knn -- python3 -u bench.py --workload knn --steps 2 --warmup 1 > "$OUT/prof.log" 2>&1
rc=$?
tail -n 3 "$OUT/tests.txt"; cat "$OUT/knn32.json" "$OUT/knn16.json"; tail -3 "$OUT/knn32.err"
echo "chain rc=$rc"
exit $rc
