#!/bin/bash
# round 4 (h): everything pending in one session -
#  tests: certified kNN (per-half lists), exact k-means assign (km_assign_p), randn (branch-free
#         table), gemm_f32t with the paired-stage barrier schedule (HEAT_GEMM_F32_PAIR=1)
#  benches: knn, kmeans (exact path: new vs round-3 kernel), gemm 8192^3 pair vs default vs hipBLASLt
#  profiles: randn kernel trace, knn issue counters
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4h"
mkdir -p "$OUT"
cd "$ROOT"
A="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests/test_gpu_kernels.py tests/test_gpu_oracle.py -m gpu \
  -k "certified or exact or threefry" > "$OUT/tests.txt" 2>&1 && \
HEAT_GEMM_F32_PAIR=1 timeout -k 10 300 $T tests/test_gpu_gemm.py tests/test_gpu_qr.py -m gpu > "$OUT/tests_pair.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py --workload knn --steps 2 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err" && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$OUT/kmeans.json" 2> "$OUT/kmeans.err" && \
HEAT_KM_ASSIGN_V1=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$OUT/kmeans_v1.json" 2> "$OUT/kmeans_v1.err" && \
timeout -k 10 200 python -u tools/microbench/gemm_bench.py 8192x8192x8192 > "$OUT/gemm_default.txt" 2>&1 && \
HEAT_GEMM_F32_PAIR=1 timeout -k 10 200 python -u tools/microbench/gemm_bench.py 8192x8192x8192 > "$OUT/gemm_pair.txt" 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_randn" -o randn -- python3 "$ROOT/tools/microbench/pmc_targets.py" randn > "$OUT/prof_randn.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace --output-format csv -d "$OUT/pmc_knn_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_A.log" 2>&1
rc=$?
cd "$ROOT"
find "$OUT" -name '*kernel_trace.csv' -delete 2>/dev/null
tail -n 2 "$OUT/tests.txt" "$OUT/tests_pair.txt"; cat "$OUT/gemm_default.txt" "$OUT/gemm_pair.txt" | cut -c1-250
echo "chain rc=$rc"
exit $rc
