# round-3 validation after the oracle checks: full GPU suite, smoke, 1-GPU bench (k-means, knn)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/t_gpu_all.txt" 2>&1 && \
timeout -k 10 120 python -u __graft_entry__.py smoke > "$OUT/smoke.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py > "$OUT/bench_1gpu.json" 2> "$OUT/bench_1gpu.err" && \
timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > "$OUT/bench_knn_1gpu.json" 2> "$OUT/bench_knn_1gpu.err"
rc=$?
tail -3 "$OUT/t_gpu_all.txt"; cat "$OUT/bench_1gpu.json" "$OUT/bench_knn_1gpu.json"
echo "chain rc=$rc"
exit $rc
