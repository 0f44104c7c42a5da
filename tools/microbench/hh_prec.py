"""Precision probe of the Householder QR's pieces on the device: the fp32 rank-K update through
hipBLASLt (torch addmm_) under float32 matmul precision "highest" and "high", the hand-written
gemm_f32t, and vtc64 (fp32 V, narrow and wide), each against an fp64 product; then the whole
Householder QR under both precision settings. One JSON line per measurement."""
import json

import torch

from heat_amd import ops
from heat_amd.ops import kernels as K


def rel(c, ref, bound):
    return float(((c.double() - ref).abs() / bound).max())


def main():
    torch.manual_seed(0)
    m, kk, n = 200_000, 256, 1024
    V = torch.randn(m, kk, device="cuda")
    X = torch.randn(kk, n, device="cuda")
    C0 = torch.randn(m, n, device="cuda")
    ref = C0.double() - V.double() @ X.double()
    bound = C0.double().abs() + V.double().abs() @ X.double().abs()
    u = 2.0 ** -24
    for prec in ("highest", "high"):
        torch.set_float32_matmul_precision(prec)
        C = C0.clone()
        C.addmm_(V, X, alpha=-1.0)
        torch.cuda.synchronize()
        print(json.dumps({"piece": "addmm_", "precision": prec, "err_units_per_k": rel(C, ref, bound) / u / kk}),
              flush=True)
    C = C0.clone()
    K.gemm_f32(V, X, out=C, accumulate=True, alpha=-1.0)
    print(json.dumps({"piece": "gemm_f32t", "err_units_per_k": rel(C, ref, bound) / u / kk}), flush=True)
    for nc in (32, 256):
        W = K.vtc64(V[:, :nc].contiguous(), C0)
        Wr = V[:, :nc].double().T @ C0.double()
        Wb = V[:, :nc].double().abs().T @ C0.double().abs()
        print(json.dumps({"piece": "vtc64", "nc": nc, "err_units_fp64": rel(W, Wr, Wb) / 2.0 ** -53 / m}),
              flush=True)
    A = torch.randn(100_000, 512, device="cuda")
    for prec in ("highest", "high"):
        torch.set_float32_matmul_precision(prec)
        Q, R = ops.householder_qr(A, 0, A.shape[0], True)
        G = Q.double().T @ Q.double()
        orth = float((G - torch.eye(G.shape[0], dtype=torch.float64, device="cuda")).abs().max())
        rec = float((Q.double() @ R.double() - A.double()).abs().max() / A.abs().max())
        print(json.dumps({"op": "householder_qr", "precision": prec, "orth": orth, "rec": rec}), flush=True)


if __name__ == "__main__":
    main()
