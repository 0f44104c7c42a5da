#!/bin/bash
# round 5 (ac): kernel trace of the flagship bench step (k = 1024): per-step sequence and durations
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5ac"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench" -o b -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --comm-ab 0 > "$OUT/bench.log" 2>&1
rc=$?
grep metric "$OUT/bench.log" | cut -c1-200
echo "chain rc=$rc"
exit $rc
