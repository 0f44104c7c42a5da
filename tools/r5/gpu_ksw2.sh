#!/bin/bash
# small-k: two-buffer wave kernel (HEAT_KS_VARIANT=w2) vs default: numerics under w2, fit loop, reference protocol
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT" TMPDIR=/tmp
OUT="$ROOT/gpurun_out/r5ksw2"; mkdir -p "$OUT"; cd "$ROOT"
HEAT_KS_VARIANT=w2 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "kmeans or lloyd or small" > "$OUT/tests.txt" 2>&1 || exit $?
for v in w w2 w w2; do
  HEAT_KS_VARIANT=$v timeout -k 10 200 python -u tools/microbench/smallk_fitloop2.py > "$OUT/fit_$v.jsonl" 2>&1 || exit $?
  HEAT_KS_VARIANT=$v timeout -k 10 300 python -u -m benchmarks.kmeans.run --case reference --trials 5 >> "$OUT/ref_$v.jsonl" 2>> "$OUT/ref.err" || exit $?
  echo "$v $(grep -o '"mean": [0-9.]*' $OUT/fit_$v.jsonl | tr '\n' ' ') ref $(grep -o '"median_s": [0-9.]*' $OUT/ref_$v.jsonl | tail -1)"
done
tail -n 1 "$OUT/tests.txt"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d "$OUT/gs_A" -o a -- python3 "$ROOT/tools/microbench/pmc_targets.py" gemm_f32s_big > "$OUT/gs_A.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU --kernel-trace --output-format csv -d "$OUT/gs_L" -o l -- python3 "$ROOT/tools/microbench/pmc_targets.py" gemm_f32s_big > "$OUT/gs_L.log" 2>&1
