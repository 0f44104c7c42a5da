#!/bin/bash
# round 4 (u): small-k k-means pass, loads two tiles ahead (default) vs one (HEAT_KS_AHEAD=1)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT"
OUT="$ROOT/gpurun_out/r4u"
mkdir -p "$OUT"
cd "$ROOT"
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_kernels.py -m gpu -k "small or kmeans" > "$OUT/tests.txt" 2>&1 && \
timeout -k 10 200 python -u tools/microbench/smallk_bench.py > "$OUT/ahead2.txt" 2>&1 && \
HEAT_KS_AHEAD=1 timeout -k 10 200 python -u tools/microbench/smallk_bench.py > "$OUT/ahead1.txt" 2>&1
rc=$?
tail -n 2 "$OUT/tests.txt"; grep -v amdgpu.ids "$OUT/ahead2.txt" "$OUT/ahead1.txt"
echo "chain rc=$rc"
exit $rc
