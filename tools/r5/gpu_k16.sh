#!/bin/bash
# 128-tile GEMM: 16-k stages / 3 workgroups per CU (HEAT_GS_K16=1) vs 32-k / 2 (default); GEMM tests both ways
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/k16; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -k "gemm or matmul" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests32.log 2>&1 || { tail -20 $O/tests32.log; exit 1; }
HEAT_GS_K16=1 timeout -k 10 400 python -u -m pytest tests -m gpu -k "gemm or matmul" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests16.log 2>&1 || { tail -20 $O/tests16.log; exit 1; }
tail -1 $O/tests32.log; tail -1 $O/tests16.log
timeout -k 10 300 python -u tools/microbench/gemm_small.py > $O/gs32.jsonl 2>&1 || exit $?
HEAT_GS_K16=1 timeout -k 10 300 python -u tools/microbench/gemm_small.py > $O/gs16.jsonl 2>&1 || exit $?
python - <<'PY'
import json
for f in ("gs32", "gs16"):
    for l in open("gpurun_out/k16/%s.jsonl" % f):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["M"], d["N"], d["K"], d.get("gemm_f32s_ms"), d.get("hipblaslt_ms"), d.get("f32s_vs_lib"))
PY
