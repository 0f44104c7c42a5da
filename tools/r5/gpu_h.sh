#!/bin/bash
# round 5 (h): split-K scan of the hand-written fp32 GEMMs vs hipBLASLt; Householder update A/B
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5h"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/microbench/gemm_splitk_scan.py > "$OUT/splitk_scan.jsonl" 2>&1 && \
timeout -k 10 900 python -u tools/microbench/hh_update_ab.py > "$OUT/hh_update_ab.jsonl" 2>&1
rc=$?
cat "$OUT/splitk_scan.jsonl" "$OUT/hh_update_ab.jsonl" | grep -v amdgpu.ids
echo "chain rc=$rc"
exit $rc
