"""Certified one-term k-means assignment vs the full fp16x3 kernel, k=1024 f=64 n=12.5M, on
diffuse (normal) data and on clustered data (points = centroid + sigma * noise)."""
import torch

from heat_amd import ops

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
n, k, f = 12_500_000, 1024, 64
C = torch.randn(k, f, device=dev, generator=g)
for sigma in (None, 0.1, 0.3, 0.5):
    if sigma is None:
        X = torch.randn(n, f, device=dev, generator=g)
    else:
        X = C[torch.randint(0, k, (n,), device=dev, generator=g)] + sigma * torch.randn(n, f, device=dev, generator=g)
    P = ops.kmeans_pack_points(X)
    res = {}
    for cert in (False, True):
        for _ in range(2):
            ops.kmeans_assign(X, C, want_mind=False, packed=P, certified=cert)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            lab, _ = ops.kmeans_assign(X, C, want_mind=False, packed=P, certified=cert)
        e1.record()
        torch.cuda.synchronize()
        res[cert] = (e0.elapsed_time(e1) / 10, lab)
    nre = int(ops.kmeans_assign.last_rechecked.item())
    agree = (res[True][1] == res[False][1]).float().mean().item()
    print(f"data={'normal' if sigma is None else f'clustered sigma={sigma}'}: full {res[False][0]:.3f} ms, "
          f"certified {res[True][0]:.3f} ms, rechecked {nre / n:.4f}, label agreement {agree:.6f}", flush=True)
    del X, P
