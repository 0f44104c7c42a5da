# round-3 GPU chain q: assign-kernel chunk-DMA prefetch A/B (HEAT_H3_DP) + kernel tests under it
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
T="python -u -m pytest -q -x --timeout 200 --timeout-method thread"
B="python -u bench.py --exact-steps 0"
HEAT_H3_DP=1 timeout -k 10 300 $T tests/test_gpu_kernels.py -k "kmeans or lasso" > "$OUT/t_dp.txt" 2>&1 && \
HEAT_H3_DP=1 timeout -k 10 200 $B > "$OUT/dp1.json" 2>/dev/null && \
timeout -k 10 200 $B > "$OUT/dp0.json" 2>/dev/null && \
HEAT_H3_DP=1 timeout -k 10 200 $B > "$OUT/dp1b.json" 2>/dev/null && \
timeout -k 10 200 $B > "$OUT/dp0b.json" 2>/dev/null
echo "chain rc=$?"
