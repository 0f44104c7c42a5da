#!/bin/bash
# round 5 (ae): Householder column steps that skip the finished panel columns (V^T V by one GEMM)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5ae"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_qr.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 400 python -u tools/microbench/hh_update_ab.py blas > "$OUT/hh_skip.jsonl" 2> "$OUT/hh_skip.err" && \
HEAT_HH_SKIP=0 timeout -k 10 400 python -u tools/microbench/hh_update_ab.py blas > "$OUT/hh_noskip.jsonl" 2> "$OUT/hh_noskip.err"
rc=$?
tail -n 1 "$OUT/tests.txt"; cat "$OUT/hh_skip.jsonl" "$OUT/hh_noskip.jsonl"
echo "chain rc=$rc"
exit $rc
