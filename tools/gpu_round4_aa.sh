#!/bin/bash
# round 4 (aa): software-pipelined cdist (cdist_pp: tile c stored between tile c+1's k-steps):
# cdist tests, bench cdist A/B (HEAT_CDIST_PIPE=1 vs 0), SUSY case A/B
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4aa"
mkdir -p "$OUT"
cd "$ROOT"
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_kernels.py tests/test_gpu_oracle.py tests/test_gpu_dist.py -m gpu -k "cdist or distance or spatial" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py --workload cdist --steps 2 --warmup 1 > "$OUT/cd1.json" 2> "$OUT/cd1.err" && \
HEAT_CDIST_PIPE=0 timeout -k 10 300 python -u bench.py --workload cdist --steps 2 --warmup 1 > "$OUT/cd0.json" 2> "$OUT/cd0.err" && \
timeout -k 10 300 python -u bench.py --workload cdist --steps 2 --warmup 1 > "$OUT/cd1b.json" 2> "$OUT/cd1b.err" && \
timeout -k 10 200 python -u -m benchmarks.distance_matrix.run --trials 5 > "$OUT/susy1.txt" 2>&1 && \
HEAT_CDIST_PIPE=0 timeout -k 10 200 python -u -m benchmarks.distance_matrix.run --trials 5 > "$OUT/susy0.txt" 2>&1
rc=$?
tail -n 2 "$OUT/tests.txt"; for f in cd1 cd0 cd1b; do python -c "import json,sys; d=json.load(open('$OUT/$f.json')); print('$f', d['ms_per_step'], d['extra'].get('cdist_ok', d['extra'].get('max_rel_err')))" 2>/dev/null || cat "$OUT/$f.json"; done; grep -h median "$OUT/susy1.txt" "$OUT/susy0.txt" | cut -c1-200
echo "chain rc=$rc"
exit $rc
