"""Small-k (k <= 16, f <= 64) fused k-means pass: assign only and assign + sums, vs HBM read time."""
import torch
from heat_amd import ops

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)


def t(fn, it=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for n, f, k in [(12_500_000, 64, 8), (12_500_000, 16, 8), (12_500_000, 64, 16), (12_500_000, 64, 3), (50_000_000, 18, 8)]:
    X = torch.randn(n, f, device=dev, generator=g)
    C = torch.randn(k, f, device=dev, generator=g)
    a = t(lambda: ops.kmeans_assign(X, C, want_mind=False))
    s = t(lambda: ops.kmeans_step_small(X, C))
    lab = ops.kmeans_assign(X, C, want_mind=False)[0]
    u = t(lambda: ops.kmeans_update(X, lab, k))
    gb = n * f * 4 / 1e9
    print(f"n={n} f={f} k={k}: assign {a:.3f} ms ({gb / a:.2f} TB/s), fused assign+sums {s:.3f} ms "
          f"({gb / s:.2f} TB/s), separate update {u:.3f} ms", flush=True)
    del X
