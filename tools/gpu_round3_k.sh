# round-3 GPU chain k: f32t pair pipeline (HEAT_GEMM_F32_PAIR=1) - GEMM tests, then A/B vs default
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
T="python -u -m pytest -q -x --timeout 200 --timeout-method thread"
S="8192x8192x8192 1250000x4096x4096 gram:1250000:4096"
HEAT_GEMM_F32_PAIR=1 timeout -k 10 400 $T tests/test_gpu_gemm.py > "$OUT/t_gemm_pair.txt" 2>&1 && \
HEAT_GEMM_F32_PAIR=1 timeout -k 10 300 python -u tools/microbench/gemm_bench.py $S --only=f32t,blas_f32 --quick > "$OUT/gemm_pair1.jsonl" 2>&1 && \
timeout -k 10 300 python -u tools/microbench/gemm_bench.py $S --only=f32t,blas_f32 --quick > "$OUT/gemm_pair0.jsonl" 2>&1
echo "chain rc=$?"
