"""Householder QR (ops.householder_qr, factor + explicit Q) of a 1.25e6 x 4096 fp32 block with the
rank-256 trailing update on hipBLASLt (HEAT_HH_UPDATE=blas, exact fp32) vs the hand-written
fp16x3 GEMM (h3: fp32-GEMM accuracy on the FP16 matrix cores) vs the exact 256-tile one (f32t); each variant in its own process (the switch is read at
import). One JSON line per variant: seconds per factorisation, ||Q^T Q - I||_max and the reconstruction
error of the first 200000 rows."""
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
qd = q.double()
orth = float((qd.T @ qd - torch.eye(n, dtype=torch.float64, device=qd.device)).abs().max())
del qd
rec = float((q[:200000].double() @ r.double() - a[:200000].double()).abs().max() / a[:200000].abs().max())
print(json.dumps({"update": os.environ["HEAT_HH_UPDATE"], "m": m, "n": n, "s": min(ts), "times": ts,
                  "orth": orth, "rec_200k_rows": rec}), flush=True)
'''

for upd in (sys.argv[1:] or ["blas", "h3", "f32t", "small"]):
    env = dict(os.environ, HEAT_HH_UPDATE=upd)
    subprocess.run([sys.executable, "-u", "-c", CHILD], env=env, timeout=400)
