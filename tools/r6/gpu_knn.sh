#!/bin/bash
# round 6: kNN screening kernel with the XCD-aligned sweep - tests, bench A/B (HEAT_H1_DEBUG=8: start
# at chunk 0 as before), L2 hit counters
set -o pipefail
OUT=gpurun_out/r6knn2; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "knn or topk" > $OUT/test.txt 2>&1 || exit 1
echo tests ok
timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_aligned.json 2> $OUT/knn_aligned.err || exit 2
HEAT_H1_DEBUG=8 timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_start0.json 2> $OUT/knn_start0.err || exit 3
timeout -k 10 200 python -u bench.py --workload knn --steps 3 --warmup 1 > $OUT/knn_aligned2.json 2> $OUT/knn_aligned2.err || exit 4
echo bench ok
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_l2 -o l2 -- python3 $ROOT/tools/microbench/pmc_targets.py knn > $ROOT/$OUT/pmc_l2.log 2>&1 || exit 5
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $ROOT/$OUT/pmc_A -o a -- python3 $ROOT/tools/microbench/pmc_targets.py knn > $ROOT/$OUT/pmc_A.log 2>&1 || exit 6
echo pmc ok
