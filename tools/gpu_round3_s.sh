#!/bin/bash
# sklearn/SciPy oracle checks on the MI355X: world of one and 2 device-buffer ranks
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_oracle.py "tests/test_gpu_dist.py" -k "oracle" > gpurun_out/oracle_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/oracle_gpu.log
exit $rc
