#!/bin/bash
# round 5 (x): Householder QR with 16-column panels (HEAT_HH_NB=16) vs 32, kernel traces
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5x"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_qr.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests32.txt" 2>&1 && \
HEAT_HH_NB=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_qr.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/tests16.txt" 2>&1 && \
timeout -k 10 600 python -u tools/microbench/hh_update_ab.py blas > "$OUT/hh32.jsonl" 2> "$OUT/hh32.err" && \
HEAT_HH_NB=16 timeout -k 10 600 python -u tools/microbench/hh_update_ab.py blas > "$OUT/hh16.jsonl" 2> "$OUT/hh16.err" && \
cd /tmp && HEAT_HH_NB=16 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nb16" -o n -- python3 "$ROOT/tools/microbench/hh_profile.py" > "$OUT/nb16.log" 2>&1
rc=$?
find "$OUT" -name '*kernel_trace.csv' -delete
tail -n 1 "$OUT/tests32.txt" "$OUT/tests16.txt"; cat "$OUT/hh32.jsonl" "$OUT/hh16.jsonl"
echo "chain rc=$rc"
exit $rc
