"""The Householder trailing-update shape C[m, N] -= V[m, 256] X[256, N] (C a column slice of the
factored matrix, row stride 4096): hipBLASLt (exact fp32 addmm), the 256-tile ``gemm_f32t`` and
the 128-tile ``gemm_f32s``, one process. Run twice with HEAT_GEMM_F32_PRELOAD=0 / 1 for the A/B of
the C-preloading accumulate path. One JSON line per shape."""
import json
import os
import time

import torch

from heat_amd.ops import kernels as K


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    torch.manual_seed(0)
    m = int(os.environ.get("UPDATE_ROWS", "1250000"))
    A = torch.randn(m, 4096, device="cuda")
    for N, Kd in ((3840, 256), (2048, 256), (768, 256), (4096, 256), (3840, 512)):
        C = A[:, 4096 - N:]
        V = torch.randn(m, Kd, device="cuda")
        X = torch.randn(Kd, N, device="cuda") * 1e-3
        ref = C.double().clone()
        ref.addmm_(V.double(), X.double(), alpha=-1.0)
        K.gemm_f32(V, X, out=C, accumulate=True, alpha=-1.0)
        err = float((C.double() - ref).abs().max())
        t_lib = timed(lambda: K._exact_addmm_(C, V, X, -1.0))
        t_f32t = timed(lambda: K.gemm_f32(V, X, out=C, accumulate=True, alpha=-1.0))
        t_s = timed(lambda: K.gemm_f32_small(V, X, out=C, accumulate=True, alpha=-1.0))
        fl = 2.0 * m * N * Kd
        print(json.dumps({"M": m, "N": N, "K": Kd, "preload": os.environ.get("HEAT_GEMM_F32_PRELOAD", "1"),
                          "hipblaslt_ms": round(t_lib, 3), "gemm_f32t_ms": round(t_f32t, 3),
                          "gemm_f32s_ms": round(t_s, 3), "f32t_vs_lib": round(t_f32t / t_lib, 3),
                          "f32s_vs_lib": round(t_s / t_lib, 3), "hipblaslt_tf": round(fl / t_lib / 1e9, 1),
                          "gemm_f32t_tf": round(fl / t_f32t / 1e9, 1), "f32t_max_abs_err": err}), flush=True)
        del V, X, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
