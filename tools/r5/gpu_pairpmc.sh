#!/bin/bash
# round 5: PMC of the pair-barrier kNN screening kernel
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5pairpmc"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
true && \
true && \
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d "$OUT/pmc_knn_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_A.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_knn_F" -o f -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_F.log" 2>&1
rc=$?
cd "$ROOT"
tail -n 3 "$OUT/tests.txt"; cut -c1-900 "$OUT/knn.json"; tail -2 "$OUT/pmc_knn_A.log"
echo "chain rc=$rc"
exit $rc
