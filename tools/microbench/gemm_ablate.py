"""Ablation of the 256-tile GEMM pipeline (``gemm_tiled.hip``): each kernel run with parts of its
stage switched off through HEAT_GEMM_ABLATE (bit 0: no DMA, 1: no wait/barrier, 2: no fragment
reads) and both f32 MFMA shapes (HEAT_GEMM_F32_SHAPE 16 / 32), each variant in a child process
(the flags are read once per process). Prints JSON lines."""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, torch
from heat_amd import ops
M, K, N = (int(v) for v in sys.argv[1].split("x"))
which = sys.argv[2]
a = torch.randn(M, K, device="cuda"); b = torch.randn(K, N, device="cuda"); c = torch.empty(M, N, device="cuda")
if which == "h3":
    pa = ops.h3_planes(a, 1); pb = ops.h3_planes(b, 0)
    fn = lambda: ops.gemm_h3_planes(pa, pb, c)
else:
    fn = lambda: ops.gemm_f32(a, b, out=c)
for _ in range(2): fn()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 5
s.record()
for _ in range(reps): fn()
e.record(); torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
print(json.dumps({"ms": ms, "tflops": 2.0 * M * N * K / ms / 1e9}))
'''


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "8192x8192x8192"
    runs = [("h3", None, a) for a in (0, 1, 2, 3, 4, 5, 7)] + \
           [("f32", sh, a) for sh in (32, 16) for a in (0, 1, 2, 4, 7)]
    for which, shp, abl in runs:
        env = dict(os.environ, HEAT_GEMM_ABLATE=str(abl))
        if shp:
            env["HEAT_GEMM_F32_SHAPE"] = str(shp)
        r = subprocess.run([sys.executable, "-c", CHILD, shape, which], env=env, capture_output=True, text=True,
                           timeout=300)
        rec = {"kernel": which, "f32_shape": shp, "ablate": abl, "shape": shape}
        if r.returncode == 0:
            rec.update(json.loads(r.stdout.strip().splitlines()[-1]))
        else:
            rec["error"] = r.stderr[-300:]
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
