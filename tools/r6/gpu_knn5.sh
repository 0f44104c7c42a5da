#!/bin/bash
# round 6: kNN screening kernel A/B - default (2 WGs/CU x 4 waves x 32 points, barrier per chunk
# pair) vs HEAT_H1_CFG=p / g (1 WG/CU x 8 waves x 32 points, barrier per 2 / 4 chunks)
set -o pipefail
OUT=gpurun_out/r6knn5; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
HEAT_H1_CFG=p timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "certified or rescore or knn_topk" > $OUT/tests_p.txt 2>&1 || exit 1
for c in def p g def p g; do
  HEAT_H1_CFG=$c timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 >> $OUT/knn.jsonl 2>> $OUT/knn.err || exit 2
done
echo ok
