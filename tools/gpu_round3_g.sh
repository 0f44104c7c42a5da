# round-3 GPU chain g: moments tests (fused epilogue, write-through hand-off), A/B and wall timing
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "moments" > "$OUT/t_moments.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/moments_ab.py > "$OUT/moments_ab.jsonl" 2> "$OUT/moments_ab.err" && \
timeout -k 10 200 python -u tools/microbench/moments_prof.py > "$OUT/moments_wall.jsonl" 2> "$OUT/moments_wall.err"
echo "chain rc=$?"
