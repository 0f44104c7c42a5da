#!/bin/bash
# kernel trace of the small-k Lloyd loop: kmeans_lloyd_small vs step + finalize
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT" TMPDIR=/tmp
OUT="$ROOT/gpurun_out/r5kstrace"; mkdir -p "$OUT"; cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o t -- python3 "$ROOT/tools/microbench/smallk_trace.py" > "$OUT/tr.log" 2>&1
