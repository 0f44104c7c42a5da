#!/bin/bash
# round 4 (l): compact-panel Householder (V^T V from the step sums): QR tests, the pieces, the
# whole 1.25e6 x 4096 QR at outer width 256 and 512
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4l"
mkdir -p "$OUT"
cd "$ROOT"
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_qr.py -m gpu > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u tools/microbench/hh_parts.py > "$OUT/parts.jsonl" 2> "$OUT/parts.err" && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh.jsonl" 2> "$OUT/hh.err" && \
HEAT_HH_OUTER=512 timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh512.jsonl" 2> "$OUT/hh512.err"
rc=$?
tail -n 3 "$OUT/tests.txt"; cat "$OUT/parts.jsonl"; grep householder "$OUT/hh.jsonl" "$OUT/hh512.jsonl"; tail -3 "$OUT/parts.err"
echo "chain rc=$rc"
exit $rc
