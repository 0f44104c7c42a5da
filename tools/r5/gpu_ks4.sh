#!/bin/bash
# small-k w2 pass: PMC passes (smallk target) + the fit loop with the Lloyd body again at the end
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT" TMPDIR=/tmp
mkdir -p "$ROOT/gpurun_out/r5ks4"
PMC_TARGETS=smallk bash "$ROOT/tools/r5/gpu_pmc.sh" || exit $?
cd "$ROOT" && timeout -k 10 200 python -u tools/microbench/smallk_fitloop2.py > gpurun_out/r5ks4/fit.jsonl 2>&1 || exit $?
grep -o '^{"[a-z_A-Z0-9]*"\|"mean": [0-9.]*' gpurun_out/r5ks4/fit.jsonl | paste - - | tr '\n' ' '
echo
timeout -k 10 300 python -u tools/microbench/gemm_small.py > gpurun_out/r5ks4/gs_prio0.jsonl 2>&1 || exit $?
HEAT_GS_PRIO=1 timeout -k 10 300 python -u tools/microbench/gemm_small.py > gpurun_out/r5ks4/gs_prio1.jsonl 2>&1 || exit $?
python - <<'PY'
import json
for f in ("gs_prio0", "gs_prio1"):
    for l in open("gpurun_out/r5ks4/%s.jsonl" % f):
        if l.startswith("{"):
            d = json.loads(l); print(f, d["M"], d["N"], d["K"], d.get("gemm_f32s_ms"), d.get("hipblaslt_ms"), d.get("f32s_vs_lib"))
PY
