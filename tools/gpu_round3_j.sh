# round-3 GPU chain j: f32t MFMA shape A/B (32x32x2 vs 16x16x4) against hipBLASLt
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
S="8192x8192x8192 1250000x4096x4096 gram:1250000:4096"
timeout -k 10 300 python -u tools/microbench/gemm_bench.py $S --only=f32t,blas_f32 --quick > "$OUT/gemm_s32.jsonl" 2>&1 && \
HEAT_GEMM_F32_SHAPE=16 timeout -k 10 300 python -u tools/microbench/gemm_bench.py $S --only=f32t,blas_f32 --quick > "$OUT/gemm_s16.jsonl" 2>&1
echo "chain rc=$?"
