#!/bin/bash
# round 6: kNN screening kernel A/B - default vs HEAT_H1_CFG=g (1 WG/CU x 8 waves, barrier per 4
# chunks) vs d / e (8 waves, groups of 2 / 3 chunks, two groups in flight)
set -o pipefail
OUT=gpurun_out/r6knn6; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
for c in d e; do
  HEAT_H1_CFG=$c timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "certified or rescore or knn_topk" > $OUT/tests_$c.txt 2>&1 || exit 1
done
for c in def g d e def g d e; do
  echo "{\"cfg\": \"$c\"}" >> $OUT/knn.jsonl
  HEAT_H1_CFG=$c timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 >> $OUT/knn.jsonl 2>> $OUT/knn.err || exit 2
done
echo ok
