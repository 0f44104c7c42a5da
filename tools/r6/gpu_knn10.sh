#!/bin/bash
# round 6: the 8-wave kNN screening form at f = 64 - tests, then bench (f = 64) vs HEAT_H1_CFG=o
set -o pipefail
OUT=gpurun_out/r6knn10; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "knn or topk or certified or rescore" > $OUT/tests.txt 2>&1 || exit 1
for c in def o def o; do
  echo "{\"cfg\": \"$c\"}" >> $OUT/knn.jsonl
  HEAT_H1_CFG=$c timeout -k 10 200 python -u bench.py --workload knn --f 64 --steps 3 --warmup 1 >> $OUT/knn.jsonl 2>> $OUT/knn.err || exit 2
done
echo "{\"cfg\": \"def f128\"}" >> $OUT/knn.jsonl
timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 >> $OUT/knn.jsonl 2>> $OUT/knn.err || exit 3
echo ok
