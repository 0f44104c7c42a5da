#!/bin/bash
# round 6: kNN screening kernel A/B - default (2 WGs/CU x 4 waves x 32 points) vs HEAT_H1_CFG=n
# (2 WGs/CU x 4 waves x 64 points)
set -o pipefail
OUT=gpurun_out/r6knn3; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
HEAT_H1_CFG=n timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_n.json 2> $OUT/knn_n.err || exit 1
timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_def.json 2> $OUT/knn_def.err || exit 2
HEAT_H1_CFG=n timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_n2.json 2> $OUT/knn_n2.err || exit 3
echo ok
