#!/bin/bash
# round 5 (l): Householder trailing-update A/B (library vs fp16x3 vs exact 256-tile), then the
# final-version PMC passes of the round-5 kernels
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5l"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/microbench/hh_update_ab.py > "$OUT/hh_ab.jsonl" 2> "$OUT/hh_ab.err" && \
PMC_TARGETS="smallk cdist_exact gemm_small gram" timeout -k 10 900 bash tools/r5/gpu_pmc.sh > "$OUT/pmc.log" 2>&1
rc=$?
cat "$OUT/hh_ab.jsonl"; tail -3 "$OUT/pmc.log"
echo "chain rc=$rc"
exit $rc
