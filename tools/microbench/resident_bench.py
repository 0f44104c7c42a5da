"""fp16x3 assign: resident-centroid kernel (HEAT_H3_RESIDENT=1) vs chunk-staged kernel (0)."""
import os
import torch
from heat_amd import ops

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
for n, f, k in [(12_500_000, 64, 1024), (12_500_000, 64, 512), (12_500_000, 64, 2048), (6_250_000, 100, 1024),
                (12_500_000, 32, 1024), (12_500_000, 64, 200)]:
    X = torch.randn(n, f, device=dev, generator=g)
    C = torch.randn(k, f, device=dev, generator=g)
    P = ops.kmeans_pack_points(X)
    for _ in range(2):
        ops.kmeans_assign(X, C, want_mind=False, packed=P)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        lab, _ = ops.kmeans_assign(X, C, want_mind=False, packed=P)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    ref = torch.cat([torch.cdist(X[i:i + 500000], C).argmin(1) for i in range(0, min(n, 2_000_000), 500000)])
    agree = (lab[: ref.shape[0]].long() == ref).float().mean().item()
    print(f"resident={os.environ.get('HEAT_H3_RESIDENT', '0')} n={n} f={f} k={k}: {ms:.3f} ms "
          f"({2 * n * k * f / ms / 1e9:.0f} TFLOP/s-equiv), agreement with torch.cdist argmin {agree:.5f}", flush=True)
    del X, P
