#!/bin/bash
# kNN pair-barrier PMC (two passes), Gram K-chunk sweep (HEAT_GRAM_KCHUNK), Gram kernel trace
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT" TMPDIR=/tmp
OUT="$ROOT/gpurun_out/r5gramk"; mkdir -p "$OUT"; cd "$ROOT"
for kc in 4096 8192 16384 32768; do
  HEAT_GRAM_KCHUNK=$kc timeout -k 10 200 python -u -m benchmarks.linalg.run --ops gram --trials 3 > "$OUT/gram_$kc.json" 2> "$OUT/gram_$kc.err" || exit $?
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/gram_trace" -o g -- python3 -m benchmarks.linalg.run --ops gram --trials 2 > "$OUT/gram_trace.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d "$OUT/pmc_knn_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_A.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_knn_F" -o f -- python3 "$ROOT/tools/microbench/pmc_targets.py" knn > "$OUT/pmc_knn_F.log" 2>&1
rc=$?
cd "$ROOT"; for kc in 4096 8192 16384 32768; do cut -c1-260 "$OUT/gram_$kc.json"; done
exit $rc
