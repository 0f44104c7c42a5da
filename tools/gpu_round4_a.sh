#!/bin/bash
# round 4 (a): cdist_p quad-transposed 16-byte store epilogue + fast randn. Microbench (store
# variants, write-bandwidth references), the affected GPU tests, kernel traces, write-bytes PMC.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4a"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 240 ./tools/microbench/cd_bench > "$OUT/cd_bench.txt" 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_oracle.py -m gpu -k "cdist or threefry or randn or knn or topk or dist" \
  > "$OUT/tests.txt" 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_randn" -o randn -- python3 "$ROOT/tools/microbench/pmc_targets.py" randn > "$OUT/prof_randn.log" 2>&1 ) && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_cdist" -o cdist -- python3 "$ROOT/tools/microbench/pmc_targets.py" cdist > "$OUT/prof_cdist.log" 2>&1 ) && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d "$OUT/pmc_cdist_w" -o w -- python3 "$ROOT/tools/microbench/pmc_targets.py" cdist > "$OUT/pmc_cdist_w.log" 2>&1 ) && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
    -d "$OUT/pmc_randn_w" -o w -- python3 "$ROOT/tools/microbench/pmc_targets.py" randn > "$OUT/pmc_randn_w.log" 2>&1 )
rc=$?
find "$OUT" -name '*kernel_trace.csv' -delete 2>/dev/null
cat "$OUT/cd_bench.txt"; tail -3 "$OUT/tests.txt"
echo "chain rc=$rc"
exit $rc
