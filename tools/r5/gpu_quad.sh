#!/bin/bash
# kNN screening kernel: one barrier per 4 chunks (HEAT_H1_CFG=q) vs per pair (default); kNN tests under q
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/quad; mkdir -p $O
HEAT_H1_CFG=q timeout -k 10 400 python -u -m pytest tests -m gpu -k "knn or topk" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
for v in pair q pair q; do
  if [ $v = q ]; then HEAT_H1_CFG=q timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 >> $O/ab.log 2>&1 || exit $?;
  else timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 >> $O/ab.log 2>&1 || exit $?; fi
  echo "$v $(grep dbg $O/ab.log | tail -1)"
done
tail -1 $O/tests.log
