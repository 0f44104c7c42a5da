# round-3 GPU chain p: fixed-order Householder panel sums - QR tests, linalg bench (Householder)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
T="python -u -m pytest -q -x --timeout 200 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_qr.py > "$OUT/t_qr.txt" 2>&1 && \
timeout -k 10 300 $T tests/test_gpu_dist.py -k "qr or householder" > "$OUT/t_qr_dist.txt" 2>&1 && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/linalg.jsonl" 2> "$OUT/linalg.err"
echo "chain rc=$?"
