#!/bin/bash
# round 4 (f): h1_topk with per-half lists of 8 - certified-kNN GPU tests, bench knn (recheck
# fraction), kernel trace + issue counters of the knn target
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4f"
mkdir -p "$OUT"
cd "$ROOT"
A="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -m gpu -k "knn or certified" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py --workload knn --steps 2 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace --output-format csv -d "$OUT/pmc_knn_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_A.log" 2>&1
rc=$?
cd "$ROOT"
find "$OUT" -name '*kernel_trace.csv' -delete 2>/dev/null
tail -3 "$OUT/tests.txt"; cut -c1-200 "$OUT/knn.json"
echo "chain rc=$rc"
exit $rc
