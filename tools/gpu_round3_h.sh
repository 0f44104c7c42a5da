# round-3 GPU chain h: assign/update overlap microbench
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
timeout -k 10 300 python -u tools/microbench/overlap_bench.py > "$OUT/overlap.jsonl" 2> "$OUT/overlap.err"
echo "chain rc=$?"
