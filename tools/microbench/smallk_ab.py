"""A/B of the small-k f = 64 kernels (HEAT_KS_VARIANT / HEAT_KS_WPC are read once per process, so
each variant runs in its own child, which prints its own JSON lines): fused assign + sums at
n = 12.5M, k = 8 / 16 / 3, per-call time and the sums against an fp64 index_add."""
import os
import subprocess
import sys

CHILD = r'''
import json, os, sys, time
import torch
from heat_amd import ops
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(12_500_000, 64, device=dev, generator=g)
tag = {"variant": os.environ["HEAT_KS_VARIANT"], "wpc": int(os.environ["HEAT_KS_WPC"])}
for k in (8, 16, 3):
    C = torch.randn(k, 64, device=dev, generator=g)
    for _ in range(3):
        ops.kmeans_step_small(X, C)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.kmeans_step_small(X, C)
    e1.record()
    torch.cuda.synchronize()
    lab, sums, counts = ops.kmeans_step_small(X, C)
    # one-hot GEMM in fp64 (index_add_ into k * 64 addresses serialises on its atomics at k = 3)
    ref = torch.nn.functional.one_hot(lab.long(), k).double().t() @ X.double()
    rec = dict(tag, k=k, ms=e0.elapsed_time(e1) / 20, sum_err=float((sums.double() - ref).abs().max()))
    print(json.dumps(rec), flush=True)
'''

for var, wpc in (("a1", "8"), ("a2", "8"), ("wave", "8"), ("wave", "9"), ("wave", "6")):
    env = dict(os.environ, HEAT_KS_VARIANT=var, HEAT_KS_WPC=wpc)
    print("# variant", var, wpc, flush=True)
    r = subprocess.run([sys.executable, "-u", "-c", CHILD], env=env, timeout=150)
    if r.returncode != 0:
        print("# child failed", r.returncode, flush=True)
        sys.exit(1)
