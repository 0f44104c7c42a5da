#!/bin/bash
# round 4 (b): restructured cdist_p (loads complete before the stores), fast randn with the host
# table: microbench, the affected GPU tests, kernel traces of the randn / cdist targets
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4b"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 240 ./tools/microbench/cd_bench > "$OUT/cd_bench.txt" 2>&1 && \
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_oracle.py -m gpu -k "cdist or threefry or randn or knn or topk or dist" \
  > "$OUT/tests.txt" 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_randn" -o randn -- python3 "$ROOT/tools/microbench/pmc_targets.py" randn > "$OUT/prof_randn.log" 2>&1 ) && \
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_cdist" -o cdist -- python3 "$ROOT/tools/microbench/pmc_targets.py" cdist > "$OUT/prof_cdist.log" 2>&1 )
rc=$?
find "$OUT" -name '*kernel_trace.csv' -delete 2>/dev/null
cat "$OUT/cd_bench.txt"; tail -3 "$OUT/tests.txt"
find "$OUT" -name '*kernel_stats.csv' -exec sh -c 'echo {}; cut -d, -f1-8 {} | head -6' \;
echo "chain rc=$rc"
exit $rc
