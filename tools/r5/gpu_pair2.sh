#!/bin/bash
# pair-barrier kNN schedule as the default: kNN/topk tests (all f, k), h1_ab default vs HEAT_H1_CFG=b, kNN bench
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/pair2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -k "knn or topk or cdist or kmeans" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 > $O/ab.log 2>&1 &&
HEAT_H1_CFG=b timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 >> $O/ab.log 2>&1 &&
timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 >> $O/ab.log 2>&1 &&
HEAT_H1_CFG=b timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 >> $O/ab.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > $O/knn.json 2> $O/knn.err
rc=$?
tail -2 $O/tests.log; grep dbg $O/ab.log; cut -c1-300 $O/knn.json
exit $rc
