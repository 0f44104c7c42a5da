#!/bin/bash
# round 5 (y): 128-tile GEMM with grouped tile order: numerics + small-GEMM table
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5y"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u tools/microbench/gemm_small.py > "$OUT/gemm_small.jsonl" 2> "$OUT/gemm_small.err"
rc=$?
tail -n 1 "$OUT/tests.txt"; python3 -c "
import json
for l in open('$OUT/gemm_small.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['M'],d['N'],d['K'],'f32s',d['gemm_f32s_ms'],'lib',d['hipblaslt_ms'],'ratio',d['f32s_vs_lib'])
"
echo "chain rc=$rc"
exit $rc
