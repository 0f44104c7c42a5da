# round-3 GPU chain r: transposed-roles cdist (vector stores) - tests, tile timing A/B
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
T="python -u -m pytest -q -x --timeout 200 --timeout-method thread"
C="python -u bench.py --workload cdist --rows 262144 --steps 3 --warmup 1"
timeout -k 10 300 $T tests/test_gpu_kernels.py -k "cdist" > "$OUT/t_cdist.txt" 2>&1 && \
timeout -k 10 200 $C > "$OUT/cd1.json" 2>/dev/null && \
HEAT_CDIST_TR=0 timeout -k 10 200 $C > "$OUT/cd0.json" 2>/dev/null && \
timeout -k 10 200 python -u -m benchmarks.distance_matrix.run --trials 5 > "$OUT/susy1.txt" 2>&1 && \
HEAT_CDIST_TR=0 timeout -k 10 200 python -u -m benchmarks.distance_matrix.run --trials 5 > "$OUT/susy0.txt" 2>&1
echo "chain rc=$?"
