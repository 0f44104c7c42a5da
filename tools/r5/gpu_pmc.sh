#!/bin/bash
# round 5: PMC passes (SQ issue / MFMA, FETCH_SIZE, WRITE_SIZE) over the round-5 kernels
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/pmc5"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
A="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
rc=0
for w in ${PMC_TARGETS:-smallk cdist_exact knn gemm_small gram}; do
  echo "== $w" 
  timeout -s KILL 150 rocprofv3 --pmc $A --kernel-trace --output-format csv -d "$OUT/${w}_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" $w > "$OUT/${w}_A.log" 2>&1 || { rc=$?; break; }
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/${w}_B" -o b -- python3 "$ROOT/tools/microbench/pmc_targets.py" $w > "$OUT/${w}_B.log" 2>&1 || { rc=$?; break; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/${w}_C" -o c -- python3 "$ROOT/tools/microbench/pmc_targets.py" $w > "$OUT/${w}_C.log" 2>&1 || { rc=$?; break; }
done
find "$OUT" -name '*kernel_trace.csv' -delete
echo "pmc rc=$rc"
exit $rc
