#!/bin/bash
# round 5 (b): exact cdist check + SUSY timing; PMC passes over ks_step64 and cdist_vx
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r5b"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_framework.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "cdist or scalar_division" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u -m benchmarks.distance_matrix.run --case susy > "$OUT/susy.txt" 2>&1 && \
HEAT_CDIST_VK64=1 timeout -k 10 200 python -u -m benchmarks.distance_matrix.run --case susy > "$OUT/susy_vk64.txt" 2>&1 && \
PMC_TARGETS="smallk cdist_exact" timeout -k 10 600 bash tools/gpu_pmc_r03.sh > "$OUT/pmc.txt" 2>&1
rc=$?
tail -n 3 "$OUT/tests.txt"; tail -2 "$OUT/susy.txt"; tail -2 "$OUT/susy_vk64.txt"; tail -3 "$OUT/pmc.txt"
echo "chain rc=$rc"
exit $rc
