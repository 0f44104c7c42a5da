# round-3 GPU chain f: moments / k-means kernel tests, moments A/B, bench, rocprof stats of the
# bench and of the check-free linalg run (matmul + QR + Householder)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
prof() {  # name timeout cmd...
  local name=$1 tmo=$2; shift 2
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$tmo" rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_$name" -o "$name" -- "$@" ) > "$OUT/prof_$name.log" 2>&1
  local rc=$?
  find "$OUT/prof_$name" -name '*kernel_trace.csv' -delete
  find "$OUT/prof_$name" -name '*.db' -delete
  return $rc
}
timeout -k 10 400 $T tests/test_gpu_kernels.py -k "kmeans or moments" > "$OUT/t_kernels.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/moments_ab.py > "$OUT/moments_ab.jsonl" 2> "$OUT/moments_ab.err" && \
timeout -k 10 300 python -u bench.py > "$OUT/bench_1gpu.json" 2> "$OUT/bench_1gpu.err" && \
timeout -k 10 200 python -u tools/microbench/moments_prof.py > "$OUT/moments_wall.jsonl" 2> "$OUT/moments_wall.err" && \
prof bench 300 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --exact-steps 0 && \
prof lin 500 python3 "$ROOT/tools/microbench/linalg_bench.py" --no-check --householder
echo "chain rc=$?"
