# round-3 GPU chain i: PMC counters of the exact fp32 GEMMs (hand-written f32t vs hipBLASLt)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d "$OUT/pmc_gemm" -o gemm -- python3 "$ROOT/tools/microbench/gemm_bench.py" 8192x8192x8192 --only=f32t,blas_f32 --quick > "$OUT/pmc_gemm.log" 2>&1
echo "chain rc=$?"
