"""Blocked Householder QR alone (for rocprofv3 kernel statistics)."""
import sys

import torch

from heat_amd import ops

m = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
torch.manual_seed(0)
A = torch.randn(m, n, device="cuda")
q, r = ops.householder_qr(A, 0, m, True)
torch.cuda.synchronize()
