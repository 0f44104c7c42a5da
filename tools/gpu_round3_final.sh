# round-3 end-of-session GPU validation: full GPU suite, smoke, bench, rocprof stats of the bench /
# check-free linalg / moments, the 1-GPU benchmark suite, then the PMC passes of the hot kernels
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
prof() {  # name timeout cmd...
  local name=$1 tmo=$2; shift 2
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$tmo" rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_$name" -o "$name" -- "$@" ) > "$OUT/prof_$name.log" 2>&1
  local rc=$?
  find "$OUT/prof_$name" -name '*kernel_trace.csv' -delete
  find "$OUT/prof_$name" -name '*.db' -delete
  return $rc
}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > "$OUT/t_gpu_all.txt" 2>&1 && \
timeout -k 10 120 python -u __graft_entry__.py smoke > "$OUT/smoke.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py > "$OUT/bench_1gpu.json" 2> "$OUT/bench_1gpu.err" && \
timeout -k 10 200 python -u tools/microbench/moments_prof.py > "$OUT/moments_wall.jsonl" 2> "$OUT/moments_wall.err" && \
prof bench 300 python3 "$ROOT/bench.py" --steps 10 --warmup 3 --exact-steps 0 && \
prof lin 500 python3 "$ROOT/tools/microbench/linalg_bench.py" --no-check --householder && \
prof mom 200 python3 "$ROOT/tools/microbench/moments_prof.py" && \
timeout -k 10 900 python3 -u -m benchmarks.run_all --gpus 1 --out "$OUT/suite_1gpu.jsonl" > "$OUT/suite.log" 2>&1 && \
bash "$ROOT/tools/gpu_pmc_r03.sh"
echo "chain rc=$?"
