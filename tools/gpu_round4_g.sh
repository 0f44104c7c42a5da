#!/bin/bash
# round 4 (g): per-half-list h1_topk and pipelined exact k-means assign (km_assign_p):
# GPU tests, bench knn (recheck fraction), bench kmeans with its exact-path timing for the new and
# the round-3 exact kernels, issue counters of the knn step
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4g"
mkdir -p "$OUT"
cd "$ROOT"
A="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_oracle.py -m gpu -k "knn or certified or kmeans or assign or threefry or randn" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py --workload knn --steps 2 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err" && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$OUT/kmeans.json" 2> "$OUT/kmeans.err" && \
HEAT_KM_ASSIGN_V1=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$OUT/kmeans_v1.json" 2> "$OUT/kmeans_v1.err" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace --output-format csv -d "$OUT/pmc_knn_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_A.log" 2>&1 && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_randn_w" -o w -- python3 "$ROOT/tools/microbench/pmc_targets.py" randn > "$OUT/pmc_randn_w.log" 2>&1
rc=$?
cd "$ROOT"
find "$OUT" -name '*kernel_trace.csv' -delete 2>/dev/null
tail -3 "$OUT/tests.txt"
echo "chain rc=$rc"
exit $rc
