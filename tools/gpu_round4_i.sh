#!/bin/bash
# round 4 (i): h1_topk with deferred (stashed) insertion: certified-kNN tests, bench knn, issue
# counters of the knn step
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4i"
mkdir -p "$OUT"
cd "$ROOT"
A="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_oracle.py -m gpu -k "knn or certified or exact" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 300 python -u bench.py --workload knn --steps 2 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err" && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace --output-format csv -d "$OUT/pmc_knn_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_A.log" 2>&1
rc=$?
cd "$ROOT"
find "$OUT" -name '*kernel_trace.csv' -delete 2>/dev/null
tail -n 3 "$OUT/tests.txt"
echo "chain rc=$rc"
exit $rc
