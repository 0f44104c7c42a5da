#!/bin/bash
# round 4 (z): randn/rand 4 elements per thread + folded Kundu constants: tests, kernel trace
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4z"
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_kernels.py tests/test_gpu_oracle.py -m gpu -k "threefry or randn or random" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_randn" -o randn -- python3 "$ROOT/tools/microbench/pmc_targets.py" randn > "$OUT/prof_randn.log" 2>&1
rc=$?
tail -n 2 "$OUT/tests.txt"; find "$OUT/prof_randn" -name "*kernel_stats.csv" -exec grep -h "tf_fill" {} \;
echo "chain rc=$rc"
exit $rc
