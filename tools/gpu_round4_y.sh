#!/bin/bash
# round 4 (y): Householder panel step: rows in flight x grid cap A/B (step scan per config)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4y"
mkdir -p "$OUT"
cd "$ROOT"
rc=0
for cfg in "1 8" "2 8" "4 8" "1 4" "2 4" "4 4" "2 2" "4 2"; do
  set -- $cfg
  HEAT_HH_ROWS=$1 HEAT_HH_BLOCKS_PER_CU=$2 timeout -k 10 120 python -u tools/microbench/hh_step_scan.py > "$OUT/scan_r$1_b$2.jsonl" 2> "$OUT/scan_r$1_b$2.err" || { rc=$?; break; }
  echo "rows=$1 blocks/cu=$2"; cat "$OUT/scan_r$1_b$2.jsonl"
done
echo "chain rc=$rc"
exit $rc
