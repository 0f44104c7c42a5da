# round-3 GPU chain n: certified assignment with sharded workgroup-aggregated lists - tests,
# clustered/diffuse microbench, bench, k-means fit benchmark
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
T="python -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "kmeans or certified" > "$OUT/t_cert.txt" 2>&1 && \
timeout -k 10 300 python -u tools/microbench/certified_assign.py > "$OUT/cert.txt" 2>&1 && \
timeout -k 10 200 python -u bench.py --exact-steps 0 > "$OUT/bench.json" 2>/dev/null && \
timeout -k 10 300 python -u -m benchmarks.kmeans.run --trials 3 > "$OUT/kmeans_fit.txt" 2>&1
echo "chain rc=$?"
