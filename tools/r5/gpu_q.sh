#!/bin/bash
# round 5 (q): kNN 2 WGs per CU, A prefetch, queue select, uniform scale; tests, bench, PMC
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5q"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "knn or topk" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py --workload knn --steps 3 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err" && \
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d "$OUT/pmc_knn_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_A.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_knn_F" -o f -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_F.log" 2>&1
rc=$?
cd "$ROOT"
tail -n 3 "$OUT/tests.txt"; cut -c1-900 "$OUT/knn.json"; tail -2 "$OUT/pmc_knn_A.log"
echo "chain rc=$rc"
exit $rc
