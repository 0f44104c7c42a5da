#!/bin/bash
# round 6: L2 behaviour of the kNN screening kernel (h1_topk): TCC hits / misses / fetch size
set -o pipefail
OUT=gpurun_out/r6knn; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_l2 -o l2 -- python3 $ROOT/tools/microbench/pmc_targets.py knn > $ROOT/$OUT/pmc_l2.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_ea -o ea -- python3 $ROOT/tools/microbench/pmc_targets.py knn > $ROOT/$OUT/pmc_ea.log 2>&1 || exit 2
echo ok
