"""The certified kNN screening kernel (ha_h1_topk) alone on 1e6 x 1e6 x 128 normal rows, timed
with device events, under HEAT_H1_DEBUG = 0 (real), 1 (no candidate selection), 2 (no chunk
barrier), 3 (neither) - the last three give invalid lists and only bound what the selection and
the barrier coupling cost. Each setting in its own process (the switch is read once)."""
import json
import os
import subprocess
import sys

CHILD = r'''
import ctypes, json, os, torch
from heat_amd import ops
from heat_amd.ops import kernels as K
L = ops.lib()
g = torch.Generator(device="cuda").manual_seed(0)
n, f, k, kp = int(os.environ.get("H1_N", "1000000")), 128, 8, 32
x = torch.randn(n, f, device="cuda", generator=g)
pk = K.kmeans_pack_points(x)
ws = torch.empty(L.ha_h1_workspace_bytes(n, f), dtype=torch.uint8, device="cuda")
dist = torch.empty((n, kp), device="cuda"); idx = torch.empty((n, kp), dtype=torch.int32, device="cuda")
cert = torch.empty(n, dtype=torch.uint8, device="cuda")
st = ctypes.c_void_p(ops.stream_ptr(x.device))
def run():
    ops.check(L.ha_h1_topk(K._ptr(pk.planes), K._ptr(pk.sx), n, f, K._ptr(x), n, x.stride(0), K._ptr(ws), k, kp,
                           K._ptr(dist), K._ptr(idx), K._ptr(cert), st), "ha_h1_topk")
run(); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); run(); run(); e1.record(); torch.cuda.synchronize()
print(json.dumps({"dbg": int(os.environ.get("HEAT_H1_DEBUG", "0")), "n": n, "ms": e0.elapsed_time(e1) / 2,
                  "certified": float(cert.float().mean())}), flush=True)
'''

for d in sys.argv[1:] or ["0", "1", "2", "3"]:
    subprocess.run([sys.executable, "-u", "-c", CHILD], env=dict(os.environ, HEAT_H1_DEBUG=d), timeout=300)
