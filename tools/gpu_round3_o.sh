# round-3 GPU chain o: per-step meta memset A/B (HEAT_H3_META_MEMSET), bench kernel profile
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
B="python -u bench.py --exact-steps 0"
timeout -k 10 200 $B > "$OUT/b0.json" 2>/dev/null && \
HEAT_H3_META_MEMSET=1 timeout -k 10 200 $B > "$OUT/b1.json" 2>/dev/null && \
timeout -k 10 200 $B > "$OUT/b0b.json" 2>/dev/null && \
HEAT_H3_META_MEMSET=1 timeout -k 10 200 $B > "$OUT/b1b.json" 2>/dev/null && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bench" -o bench -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --exact-steps 0 > "$OUT/prof_bench.log" 2>&1 ) && \
find "$OUT/prof_bench" -name '*kernel_trace.csv' -delete
echo "chain rc=$?"
