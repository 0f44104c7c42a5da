"""One Householder factorisation + explicit Q of a 1.25e6 x 4096 fp32 block (ops.householder_qr),
for a kernel-trace profile of the trailing-update variant in HEAT_HH_UPDATE (after a small warm-up)."""
import os
import time

import torch

from heat_amd import ops

torch.manual_seed(0)
m, n = int(os.environ.get("HH_M", "1250000")), int(os.environ.get("HH_N", "4096"))
a = torch.randn(m, n, device="cuda")
ops.householder_qr(a[:200000, :1024].contiguous(), 0, 200000, True)
torch.cuda.synchronize()
t0 = time.perf_counter()
q, r = ops.householder_qr(a, 0, m, True)
torch.cuda.synchronize()
print(os.environ.get("HEAT_HH_UPDATE"), time.perf_counter() - t0, flush=True)
