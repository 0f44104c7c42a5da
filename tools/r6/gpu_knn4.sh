#!/bin/bash
# round 6: persistent kNN screening grid with the per-XCD-group sync - tests, A/B, L2 counters
set -o pipefail
OUT=gpurun_out/r6knn4; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "knn or topk" > $OUT/test.txt 2>&1 || exit 1
echo tests ok
timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_sync128.json 2> $OUT/knn_sync128.err || exit 2
HEAT_H1_SYNC=0 timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_nosync.json 2> $OUT/knn_nosync.err || exit 3
HEAT_H1_PERSIST=0 timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_orig.json 2> $OUT/knn_orig.err || exit 4
HEAT_H1_SYNC=32 timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_sync32.json 2> $OUT/knn_sync32.err || exit 5
echo bench ok
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_l2 -o l2 -- python3 $ROOT/tools/microbench/pmc_targets.py knn > $ROOT/$OUT/pmc_l2.log 2>&1 || exit 6
echo pmc ok
