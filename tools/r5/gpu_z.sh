#!/bin/bash
# round 5 (z): kernel trace of the reference k-means protocol (k = 8, 30 iterations, 1.25e7 x 64)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5z"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ref" -o r -- python3 -m benchmarks.kmeans.run --case reference --trials 3 > "$OUT/ref.log" 2>&1
rc=$?
tail -3 "$OUT/ref.log"
echo "chain rc=$rc"
exit $rc
