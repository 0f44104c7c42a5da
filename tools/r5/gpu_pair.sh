#!/bin/bash
# pair-barrier A/B of the certified kNN screening kernel (HEAT_H1_CFG=p) vs default, then the kNN tests under p
set -o pipefail
export PYTHONPATH=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 > gpurun_out/pair_def.log 2>&1 &&
HEAT_H1_CFG=p timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 2 > gpurun_out/pair_p.log 2>&1 &&
timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 >> gpurun_out/pair_def.log 2>&1 &&
HEAT_H1_CFG=p timeout -k 10 300 python -u tools/microbench/h1_ab.py 0 >> gpurun_out/pair_p.log 2>&1 &&
HEAT_H1_CFG=p timeout -k 10 400 python -u -m pytest tests -m gpu -k "knn or topk" -x -q --timeout 120 --timeout-method thread > gpurun_out/pair_tests.log 2>&1
rc=$?
cat gpurun_out/pair_def.log gpurun_out/pair_p.log; tail -3 gpurun_out/pair_tests.log
exit $rc
