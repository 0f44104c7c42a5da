#!/bin/bash
# round 6: the 1-GPU benchmark suite with the same-process torch comparators (benchmarks/run_all.py), one benchmark per step, with a
# heartbeat line every minute (the run prints its results only when a benchmark ends)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r6suite"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
rc=0
for b in ${SUITE_LIST:-kmeans kmeans_reference distance_matrix knn statistical_moments lasso linalg linalg_high}; do
  echo "== $b $(date +%T)"
  timeout -k 10 900 python -u -m benchmarks.run_all --gpus 1 --only $b --out "$OUT/suite.jsonl" --timeout 880 > "$OUT/$b.log" 2>&1 || { rc=$?; echo "$b failed rc=$rc"; break; }
done
kill $HB
wc -l "$OUT/suite.jsonl"
echo "chain rc=$rc"
exit $rc
