"""QR of the per-GPU slice of the linalg north star (1.25e6 x 4096 fp32, = 1e7 x 4096 on 8 GPUs):
CholeskyQR2 on a well-conditioned matrix vs blocked Householder (csrc/householder.hip) on a
cond = 1e10 one, with the orthogonality ||Q^T Q - I||_max of each. JSON lines."""
import json
import sys
import time

import torch

import heat_amd as ht
from heat_amd import ops


def gen(m, n, cond, seed):
    torch.manual_seed(seed)
    V, _ = torch.linalg.qr(torch.randn(n, n, device="cuda", dtype=torch.float64))
    s = torch.logspace(0, -torch.log10(torch.tensor(float(cond))).item(), n, device="cuda", dtype=torch.float64)
    B = (s.unsqueeze(1) * V.T).float()
    A = torch.empty(m, n, device="cuda")
    step = 1 << 18
    for r0 in range(0, m, step):
        A[r0: r0 + step] = torch.randn(min(step, m - r0), n, device="cuda") @ B
    return A


def orth(q):
    n = q.shape[1]
    return (q.T.double() @ q.double() - torch.eye(n, device=q.device, dtype=torch.float64)).abs().max().item()


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    ht.use_device("gpu")
    for cond in (1e2, 1e10):
        A = gen(m, n, cond, 1)
        X = ht.array(A, is_split=None)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        q, r = ht.linalg.qr(X, mode="reduced")
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res = {"m": m, "n": n, "cond": cond, "qr_s": dt, "orth": orth(q.larray)}
        del q, r
        torch.cuda.empty_cache()
        t0 = time.perf_counter()
        q2, r2 = ops.householder_qr(A, 0, m, True)
        torch.cuda.synchronize()
        res["householder_s"] = time.perf_counter() - t0
        res["householder_orth"] = orth(q2)
        print(json.dumps(res), flush=True)
        del q2, r2, A, X
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
