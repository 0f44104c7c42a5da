"""k-means centroid update (counting sort + gather): HEAT_KU_GATHER4=1 (16-byte gathers) vs 0."""
import os
import torch
from heat_amd import ops

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
for n, f, k in [(12_500_000, 64, 1024), (12_500_000, 128, 1024), (12_500_000, 64, 64)]:
    X = torch.randn(n, f, device=dev, generator=g)
    lab = torch.randint(0, k, (n,), device=dev, generator=g, dtype=torch.int32)
    for _ in range(2):
        ops.kmeans_update(X, lab, k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        s, c = ops.kmeans_update(X, lab, k)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    ref = torch.zeros(k, f, dtype=torch.float64, device=dev).index_add_(0, lab.long(), X.double())
    err = ((s.double() - ref).abs().max() / ref.abs().max()).item()
    print(f"gather4={os.environ.get('HEAT_KU_GATHER4', '1')} n={n} f={f} k={k}: {ms:.3f} ms "
          f"({n * f * 4 / ms / 1e9:.2f} TB/s), rel err {err:.2e}", flush=True)
    del X
