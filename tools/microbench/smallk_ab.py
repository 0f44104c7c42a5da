"""A/B of the small-k f = 64 kernels in one process (HEAT_KS_VARIANT / HEAT_KS_WPC are read once
per process, so each variant runs in its own child): fused assign + sums at n = 12.5M, k = 8."""
import json
import os
import subprocess
import sys

CHILD = r'''
import torch, json
from heat_amd import ops
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(12_500_000, 64, device=dev, generator=g)
res = {}
for k in (8, 16, 3):
    C = torch.randn(k, 64, device=dev, generator=g)
    for _ in range(3):
        ops.kmeans_step_small(X, C)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.kmeans_step_small(X, C)
    e1.record()
    torch.cuda.synchronize()
    res["k%d_ms" % k] = e0.elapsed_time(e1) / 20
    lab, sums, counts = ops.kmeans_step_small(X, C)
    ref = torch.zeros(k, 64, dtype=torch.float64, device=dev).index_add_(0, lab.long(), X.double())
    res["k%d_sum_err" % k] = float((sums.double() - ref).abs().max())
print(json.dumps(res))
'''

for var, wpc in (("a1", "8"), ("a2", "8"), ("wave", "8"), ("wave", "9"), ("wave", "6")):
    env = dict(os.environ, HEAT_KS_VARIANT=var, HEAT_KS_WPC=wpc)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    rec = {"variant": var, "wpc": int(wpc)}
    rec.update(json.loads(line[-1]) if line else {"error": out.stderr[-500:]})
    print(json.dumps(rec), flush=True)
