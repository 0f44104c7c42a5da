#!/bin/bash
# 128-tile GEMM with the automatic 16-k / 32-k stage choice: GEMM / matmul / QR tests, microbench
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/k16b; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -k "gemm or matmul or qr or householder or gram or linalg" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/microbench/gemm_small.py > $O/gs_auto.jsonl 2>&1 || exit $?
python - <<'PY'
import json
for l in open("gpurun_out/k16b/gs_auto.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print("auto", d["M"], d["N"], d["K"], d.get("gemm_f32s_ms"), d.get("hipblaslt_ms"), d.get("f32s_vs_lib"))
PY
