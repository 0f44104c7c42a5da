"""Householder QR (ops.householder_qr, factor + explicit Q) of a 1.25e6 x 4096 fp32 block with the
rank-256 trailing update on hipBLASLt (HEAT_HH_UPDATE=blas) vs the hand-written 128-tile GEMM
(small) vs the 256-tile one (f32t); each variant in its own process (the switch is read at
import). One JSON line per variant: seconds per factorisation and the orthogonality error."""
import json
import os
import subprocess
import sys
import time

CHILD = r'''
import json, os, time, torch
from heat_amd import ops
torch.manual_seed(0)
m, n = int(os.environ.get("HH_M", "1250000")), int(os.environ.get("HH_N", "4096"))
a = torch.randn(m, n, device="cuda")
ops.householder_qr(a[:200000, :1024].contiguous(), 0, 200000, True)   # warm-up (kernels, allocator)
torch.cuda.synchronize()
ts = []
for _ in range(2):
    t0 = time.perf_counter()
    q, r = ops.householder_qr(a, 0, m, True)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
s = torch.linalg.svdvals(q[:, :256].double().T @ q[:, :256].double())
print(json.dumps({"update": os.environ["HEAT_HH_UPDATE"], "m": m, "n": n, "s": min(ts), "times": ts,
                  "orth_256": float((s - 1).abs().max())}), flush=True)
'''

for upd in ("blas", "small", "f32t"):
    env = dict(os.environ, HEAT_HH_UPDATE=upd)
    subprocess.run([sys.executable, "-u", "-c", CHILD], env=env, timeout=400)
