#!/bin/bash
# round 6: gemm_f32m tile / barrier-group variants (A/B) - layout / update tests, then the square + update microbench
set -o pipefail
OUT=gpurun_out/${R6V_DIR:-r6v}; mkdir -p $OUT
ROOT=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "mid or layouts" > $OUT/tests.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/microbench/gemm_mid.py > $OUT/gemm_mid.jsonl 2> $OUT/gemm_mid.err || exit 2
echo ok
