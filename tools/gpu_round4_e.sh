#!/bin/bash
# round 4 (e): where the certified kNN step spends its time (kernel trace of the knn target) and
# the PMC issue counters of h1_topk / h3_topk_p; bench knn JSON with the recheck fraction
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4e"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_knn" -o knn -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/prof_knn.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace --output-format csv -d "$OUT/pmc_knn_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_A.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $A --kernel-trace --output-format csv -d "$OUT/pmc_topk_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" topk > "$OUT/pmc_topk_A.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/pmc_randn_w" -o w -- python3 "$ROOT/tools/microbench/pmc_targets.py" randn > "$OUT/pmc_randn_w.log" 2>&1 && \
cd "$ROOT" && timeout -k 10 300 python -u bench.py --workload knn --steps 2 --warmup 1 > "$OUT/knn.json" 2> "$OUT/knn.err"
rc=$?
cd "$ROOT"
find "$OUT" -name '*kernel_trace.csv' -delete 2>/dev/null
find "$OUT" -name '*kernel_stats.csv' -exec sh -c 'echo {}; cut -d, -f1-4 {} | head -12' \;
cut -c1-200 "$OUT/knn.json"
echo "chain rc=$rc"
exit $rc
