"""Per-iteration device time of the k-means Lloyd step as the fit loop runs it
(KMeans._centroid_step, k = 8, 1.25e7 x 64): the reference protocol's trace shows the fused pass
alternating 580 / 710 us between iterations while back-to-back calls with fixed buffers do not."""
import json

import torch

import heat_amd as ht

ht.use_device("gpu")
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn(12_500_000, 64, device="cuda", generator=g)
km = ht.cluster.KMeans(n_clusters=8, init="random", max_iter=30, tol=None, random_state=5)
C = X[:8].clone()
for _ in range(3):
    C, _ = km._centroid_step(X, C, None, False)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
ev[0].record()
for i in range(40):
    C, lab = km._centroid_step(X, C, None, False)
    ev[i + 1].record()
torch.cuda.synchronize()
print(json.dumps({"centroid_step_ms": [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(40)]}), flush=True)
# the same with the labels kept alive one iteration longer (as the fit loop keeps _last_labels)
keep = None
ev[0].record()
for i in range(40):
    C, lab = km._centroid_step(X, C, None, False)
    keep = lab
    ev[i + 1].record()
torch.cuda.synchronize()
print(json.dumps({"keep_labels_ms": [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(40)]}), flush=True)
