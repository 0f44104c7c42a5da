"""Kernel-trace target: 30 Lloyd steps through kmeans_lloyd_small, then 30 through
kmeans_step_small + kmeans_finalize (k = 8, 1.25e7 x 64), separated by a 50 ms idle gap, so a
rocprofv3 --kernel-trace run shows per-kernel durations and gaps of both loops
(tools/r5/gpu_kstrace.sh + the summary at the end of this file's run)."""
import time

import torch

from heat_amd import ops

g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn(12_500_000, 64, device="cuda", generator=g)
C0 = X[:8].clone()


def lloyd(C):
    return ops.kmeans_lloyd_small(X, C)[1]


def split(C):
    _, s, c = ops.kmeans_step_small(X, C)
    return ops.kmeans_finalize(None, C, sums=s, counts=c)[0]


for body in (lloyd, split, lloyd, split):
    C = C0.clone()
    for _ in range(30):
        C = body(C)
    torch.cuda.synchronize()
    time.sleep(0.05)
print("done")
