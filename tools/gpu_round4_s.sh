#!/bin/bash
# round 4 (s): sliced fp32-MFMA V^T C (1024-row slices), hh_step back to 1 row in flight: QR tests, precision probe,
# whole Householder QR at 1.25e6 x 4096, kernel trace of the Householder QR
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4s"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_qr.py -m gpu > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u tools/microbench/hh_prec.py > "$OUT/prec.jsonl" 2> "$OUT/prec.err" && timeout -k 10 300 python -u tools/microbench/hh_parts.py > "$OUT/parts.jsonl" 2> "$OUT/parts.err" && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh.jsonl" 2> "$OUT/hh.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o hh -- python3 -u tools/microbench/hh_prof.py 1250000 4096 > "$OUT/prof.log" 2>&1
rc=$?
tail -n 3 "$OUT/tests.txt"; cat "$OUT/prec.jsonl" "$OUT/parts.jsonl"; grep householder "$OUT/hh.jsonl"; tail -3 "$OUT/hh.err"
echo "chain rc=$rc"
exit $rc
