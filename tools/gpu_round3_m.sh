# round-3 GPU chain m: assign-kernel fragment prefetch A/B (HEAT_H3_PF), short-row moments pipe
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
T="python -u -m pytest -q -x --timeout 200 --timeout-method thread"
HEAT_H3_PF=1 timeout -k 10 300 $T tests/test_gpu_kernels.py -k "kmeans or moments" > "$OUT/t_pf.txt" 2>&1 && \
HEAT_H3_PF=1 timeout -k 10 200 python -u bench.py --exact-steps 0 > "$OUT/bench_pf1.json" 2>/dev/null && \
timeout -k 10 200 python -u bench.py --exact-steps 0 > "$OUT/bench_pf0.json" 2>/dev/null && \
HEAT_H3_PF=1 timeout -k 10 200 python -u bench.py --exact-steps 0 > "$OUT/bench_pf1b.json" 2>/dev/null && \
timeout -k 10 200 python -u bench.py --exact-steps 0 > "$OUT/bench_pf0b.json" 2>/dev/null && \
timeout -k 10 200 python -u tools/microbench/moments_prof.py > "$OUT/moments_wall.jsonl" 2> "$OUT/moments_wall.err"
echo "chain rc=$?"
