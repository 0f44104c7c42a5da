#!/bin/bash
# round 4 (x): parallel fixed-order tails of the Householder panel kernels: QR tests, step scan,
# whole Householder QR
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4x2"
mkdir -p "$OUT"
cd "$ROOT"
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_qr.py -m gpu > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/hh_step_scan.py > "$OUT/scan.jsonl" 2> "$OUT/scan.err" && \
timeout -k 10 300 python -u tools/microbench/linalg_bench.py --householder > "$OUT/hh.jsonl" 2> "$OUT/hh.err" && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o hh -- python3 -u tools/microbench/hh_prof.py 1250000 4096 > "$OUT/prof.log" 2>&1
rc=$?
tail -n 2 "$OUT/tests.txt"; cat "$OUT/scan.jsonl"; grep householder "$OUT/hh.jsonl"; tail -2 "$OUT/hh.err"
echo "chain rc=$rc"
exit $rc
