"""Per-call durations of the fused small-k pass (k = 8, 1.25e7 x 64) called back to back with the
same centroids and the same output buffers (device events per call): is the odd / even
alternation seen in the reference protocol's trace (580 vs 710 us) in the kernel or the caller?"""
import ctypes
import json

import torch

from heat_amd import ops
from heat_amd.ops import kernels as K

L = ops.lib()
g = torch.Generator(device="cuda").manual_seed(0)
n, f, k = 12_500_000, 64, 8
X = torch.randn(n, f, device="cuda", generator=g)
C = X[:k].clone()
ncu = ops.num_cus(X.device)
labels = torch.empty(n, dtype=torch.int32, device="cuda")
ws = torch.empty(L.ha_ks_workspace_floats(k, ncu), device="cuda")
sums = torch.empty((k, f), device="cuda")
counts = torch.empty(k, device="cuda")
st = ctypes.c_void_p(ops.stream_ptr(X.device))


def one():
    ops.check(L.ha_ks_step(K._ptr(X), n, f, f, K._ptr(C), k, f, K._ptr(labels), None, K._ptr(sums), K._ptr(counts),
                           K._ptr(ws), ncu, st), "ha_ks_step")


for _ in range(3):
    one()
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
ev[0].record()
for i in range(40):
    one()
    ev[i + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(40)]
print(json.dumps({"same_buffers_ms": [round(x, 3) for x in ms]}), flush=True)
# with a fresh labels tensor per call (what the Python path does)
ev[0].record()
for i in range(40):
    labels = torch.empty(n, dtype=torch.int32, device="cuda")
    one()
    ev[i + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(40)]
print(json.dumps({"fresh_labels_ms": [round(x, 3) for x in ms]}), flush=True)
# alternating between two labels buffers / two workspaces (what a fit loop that keeps the last
# labels alive gets from the caching allocator)
lab2 = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]
ws2 = [torch.empty_like(ws) for _ in range(2)]
for name, alt_l, alt_w in (("alt_labels_ms", True, False), ("alt_workspace_ms", False, True)):
    ev[0].record()
    for i in range(40):
        labels = lab2[i & 1] if alt_l else labels
        ws = ws2[i & 1] if alt_w else ws
        one()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(40)]
    print(json.dumps({name: [round(x, 3) for x in ms]}), flush=True)
# alternating centroid sets (data dependence of the kernel's time?)
C0 = C.clone()
C1 = X[1000:1000 + k].clone()
Cfit = None
ev[0].record()
for i in range(40):
    C = C0 if i % 2 == 0 else C1
    one()
    ev[i + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(40)]
print(json.dumps({"alt_centroids_ms": [round(x, 3) for x in ms]}), flush=True)
# converged centroids (a fit's final state) repeated
# the fit loop itself: 30 iterations of KMeans(8).fit, per-step events via the profiler-free path
import heat_amd as ht
ht.use_device("gpu")
x = ht.array(X, split=0)
km = ht.cluster.KMeans(n_clusters=8, init="random", max_iter=30, tol=None, random_state=5)
km.fit(x)
torch.cuda.synchronize()
import time
t0 = time.perf_counter()
km = ht.cluster.KMeans(n_clusters=8, init="random", max_iter=30, tol=None, random_state=5)
km.fit(x)
torch.cuda.synchronize()
print(json.dumps({"fit_30_ms": round((time.perf_counter() - t0) * 1e3, 3)}), flush=True)
C = km.cluster_centers_.larray.float().contiguous()
ev[0].record()
for i in range(40):
    one()
    ev[i + 1].record()
torch.cuda.synchronize()
ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(40)]
print(json.dumps({"converged_centroids_ms": [round(x, 3) for x in ms]}), flush=True)
