#!/bin/bash
# last check of the round: kNN / top-k / k-means GPU tests at the defaults, smoke, kNN bench
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/last; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -k "knn or topk or kmeans or lloyd or small or cdist" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > $O/knn.json 2> $O/knn.err || exit $?
tail -1 $O/tests.log; tail -1 $O/smoke.txt; cut -c1-200 $O/knn.json
