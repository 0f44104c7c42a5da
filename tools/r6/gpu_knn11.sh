#!/bin/bash
# round 6: kNN 12-entry half lists (HEAT_H1_CFG=k) vs the 16-entry default - tests, bench
set -o pipefail
OUT=gpurun_out/r6knn11; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
HEAT_H1_CFG=k timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "knn or topk or certified or rescore" > $OUT/tests_k.txt 2>&1 || exit 1
for c in def k def k; do
  echo "{\"cfg\": \"$c\"}" >> $OUT/knn.jsonl
  HEAT_H1_CFG=$c timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 >> $OUT/knn.jsonl 2>> $OUT/knn.err || exit 2
done
echo ok
