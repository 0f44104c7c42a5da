#!/bin/bash
# oracle checks on the GPU (world of one + 2 device ranks), then the fused top-k at 1e6 x 1e6 x 128
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_oracle.py "tests/test_gpu_dist.py" -k "oracle" > gpurun_out/oracle_gpu.log 2>&1 && \
timeout -k 10 300 python -u tools/microbench/topk_bench.py > gpurun_out/topk_bench.jsonl 2> gpurun_out/topk_bench.err
rc=$?
tail -4 gpurun_out/oracle_gpu.log; cat gpurun_out/topk_bench.jsonl; tail -3 gpurun_out/topk_bench.err
exit $rc
