"""Householder QR accuracy per V^T C variant (HEAT_HH_VTC = f64 | f32s, HEAT_VTC_KCHUNK) on the
ill-conditioned test matrix of tests/test_gpu_qr.py (60000 x 640, cond 1e8) and a random
200000 x 1024 block, next to LAPACK-style fp32 QR (torch.linalg.qr: rocSOLVER on the device, LAPACK
sgeqrf on the host) of the same matrices. Each variant in its own process (the switches are read
at import). One JSON line per (variant, matrix)."""
import json
import os
import subprocess
import sys

import torch


def ill(m, n, cond, seed):
    g = torch.Generator().manual_seed(seed)
    G = torch.randn(m, n, generator=g, dtype=torch.float64)
    V, _ = torch.linalg.qr(torch.randn(n, n, generator=g, dtype=torch.float64))
    s = torch.logspace(0, -torch.log10(torch.tensor(cond)).item(), n, dtype=torch.float64)
    return ((G * s) @ V.T).float()


def errs(a, q, r):
    Q = q.double()
    n = Q.shape[1]
    orth = (Q.T @ Q - torch.eye(n, dtype=torch.float64, device=Q.device)).abs().max().item()
    rec = (Q @ r.double() - a.double()).abs().max().item() / a.abs().max().item()
    return orth, rec


def mats():
    torch.manual_seed(0)
    return {"ill_60000x640": ill(60_000, 640, 1e8, 9), "randn_200000x1024": torch.randn(200_000, 1024)}


def child(tag):
    from heat_amd import ops

    for name, a in mats().items():
        ad = a.cuda()
        q, r = ops.householder_qr(ad, 0, a.shape[0], True)
        orth, rec = errs(ad, q, r)
        print(json.dumps({"variant": tag, "matrix": name, "orth": orth, "rec": rec}), flush=True)


def main():
    if len(sys.argv) > 1:
        child(sys.argv[1])
        return
    for name, a in mats().items():
        ad = a.cuda()
        q, r = torch.linalg.qr(ad)
        orth, rec = errs(ad, q, r)
        print(json.dumps({"variant": "torch.linalg.qr fp32 (device)", "matrix": name, "orth": orth, "rec": rec}),
              flush=True)
        q, r = torch.linalg.qr(a)
        orth, rec = errs(a, q, r)
        print(json.dumps({"variant": "torch.linalg.qr fp32 (host LAPACK)", "matrix": name, "orth": orth,
                          "rec": rec}), flush=True)
    for tag, env in (("f64", {"HEAT_HH_VTC": "f64"}), ("f32s_4096", {"HEAT_HH_VTC": "f32s"}),
                     ("f32s_1024", {"HEAT_HH_VTC": "f32s", "HEAT_VTC_KCHUNK": "1024"}),
                     ("f32s_512", {"HEAT_HH_VTC": "f32s", "HEAT_VTC_KCHUNK": "512"})):
        subprocess.run([sys.executable, "-u", __file__, tag], env=dict(os.environ, **env), check=True, timeout=240)


if __name__ == "__main__":
    main()
