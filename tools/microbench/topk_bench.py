"""Fused nearest-neighbour reduction at the distance-matrix benchmark size: ``spatial.cdist_topk``
of 1e6 x 128 queries against 1e6 x 128 points (the 4 TB fp32 distance matrix is never formed),
k = 1 and 8, fp32 on one GPU. Prints one JSON line per k: seconds, fp32-equivalent TFLOP/s
(2 n m f), and a recomputed check of 256 random queries against torch."""
import json
import time

import torch

import heat_amd as ht

ht.use_device("gpu")
n, f = 1_000_000, 128
X = ht.random.randn(n, f, split=0)
Y = ht.random.randn(n, f, split=0)
for k in (1, 8):
    ht.spatial.cdist_topk(X[:4096], Y, k)                  # warm-up (pack, allocator)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d, i = ht.spatial.cdist_topk(X, Y, k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    q = torch.randint(0, n, (256,), device=X.larray.device)
    ref = torch.cdist(X.larray[q].double(), Y.larray.double())
    rd, ri = torch.topk(ref, k, dim=1, largest=False)
    agree = float((i.larray[q] == ri).float().mean())
    derr = float(((d.larray[q].double() - rd).abs() / rd.clamp(min=1e-6)).max())
    print(json.dumps({"op": "cdist_topk", "n": n, "m": n, "f": f, "k": k, "seconds": dt,
                      "tflops_fp32_equiv": 2.0 * n * n * f / dt / 1e12, "index_agreement": agree,
                      "max_rel_dist_err": derr}), flush=True)
