#!/bin/bash
# small-k w2 pass: PMC passes (smallk target) + the fit loop with the Lloyd body again at the end
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
export PYTHONPATH="$ROOT" TMPDIR=/tmp
mkdir -p "$ROOT/gpurun_out/r5ks4"
PMC_TARGETS=smallk bash "$ROOT/tools/r5/gpu_pmc.sh" || exit $?
cd "$ROOT" && timeout -k 10 200 python -u tools/microbench/smallk_fitloop2.py > gpurun_out/r5ks4/fit.jsonl 2>&1 || exit $?
grep -o '^{"[a-z_A-Z0-9]*"\|"mean": [0-9.]*' gpurun_out/r5ks4/fit.jsonl | paste - - | tr '\n' ' '
