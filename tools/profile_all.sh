#!/bin/bash
# Kernel-level profiles (rocprofv3 --kernel-trace --stats, CSV) of every benchmark workload, plus
# the 1-GPU benchmark suite results. Run on the GPU box from the repo root; outputs land in
# gpurun_out/prof_<name>/ and gpurun_out/suite_1gpu.jsonl (copy summaries into profiles/).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
run() {  # name timeout cmd...
  local name=$1 tmo=$2; shift 2
  echo "=== $name"
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$tmo" rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_$name" -- "$@" ) > "$OUT/prof_$name.log" 2>&1
  local rc=$?
  grep -h '^{' "$OUT/prof_$name.log" | cut -c1-300
  echo "=== $name rc=$rc"
  return $rc
}
run kmeans 300 python3 "$ROOT/bench.py" --steps 10 --warmup 2 &&
run kmeans_reference 300 python3 -m benchmarks.kmeans.run --case reference --trials 2 &&
run knn 300 python3 "$ROOT/tools/microbench/knn_bench.py" &&
run linalg_high 400 python3 -m benchmarks.linalg.run --trials 1 --precision high &&
run kmeans_exact 300 python3 -m benchmarks.kmeans.run --precision exact --trials 1 --iterations 5 &&
run dist_susy 300 python3 -m benchmarks.distance_matrix.run --trials 3 &&
run dist_tile 300 python3 "$ROOT/bench.py" --workload cdist --rows 262144 --steps 2 --warmup 1 &&
run moments 300 python3 -m benchmarks.statistical_moments.run --trials 5 &&
run lasso 300 python3 -m benchmarks.lasso.run --trials 3 &&
run qr 400 python3 -m benchmarks.linalg.run --trials 1 &&
( timeout -k 10 900 python3 -m benchmarks.run_all --gpus 1 --out "$OUT/suite_1gpu.jsonl" > "$OUT/suite.log" 2>&1; echo "suite rc=$?" )
