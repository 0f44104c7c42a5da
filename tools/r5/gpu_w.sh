#!/bin/bash
# round 5 (w): kernel-trace profiles of the Householder QR with the library vs the fp16x3 rank update
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5w"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
HEAT_HH_UPDATE=blas timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/blas" -o b -- python3 "$ROOT/tools/microbench/hh_profile.py" > "$OUT/blas.log" 2>&1 && \
HEAT_HH_UPDATE=h3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/h3" -o h -- python3 "$ROOT/tools/microbench/hh_profile.py" > "$OUT/h3.log" 2>&1 && \
cd "$ROOT" && timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
find "$OUT" -name '*kernel_trace.csv' -delete
grep -h "^blas\|^h3" "$OUT"/*.log; cut -c1-250 "$OUT/bench.json"
echo "chain rc=$rc"
exit $rc
