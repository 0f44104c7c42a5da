#!/bin/bash
# round 6, call o: the Householder update shapes on the 64 x 64 tile
set -o pipefail
OUT=gpurun_out/r6o; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
GM_SHAPES=upd timeout -k 10 300 python tools/microbench/gemm_mid.py > $OUT/gemm_mid_upd.jsonl 2>&1 || exit 1
HEAT_GM64_MAXK=256 timeout -k 10 300 python tools/microbench/hh_update_ab.py small > $OUT/hh_k256.jsonl 2>&1 || exit 2
echo ok
