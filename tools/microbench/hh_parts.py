"""Pieces of the blocked Householder QR at the north-star shape (1.25e6 x 4096 fp32), timed alone:
  * one 32-column panel (hh_colsums + 32 hh_step launches) on a column slice of the full matrix
    (row pitch 4096) vs the same panel in a compact m x 32 buffer (row pitch 32);
  * the trailing update C -= V X (K = 256, N = 3840) on gemm_f32t vs hipBLASLt (torch addmm_);
    the inner panel update (K = 32, N = 224, C a column slice of the matrix) the same way;
  * W = V^T C (nc = 256, N = 3840) on vtc64 (fp64 matrix cores).
One JSON line per measurement."""
import ctypes
import json
import sys
import time

import torch

from heat_amd import ops
from heat_amd.ops import kernels as K


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
    n = 4096
    L = ops.lib()
    torch.manual_seed(0)
    A = torch.randn(m, n, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    nb = L.ha_hh_nb()
    slen = L.ha_hh_slen()
    hpart = torch.empty(max(1, L.ha_hh_part_len(m)), dtype=torch.float64, device="cuda")
    hcnt = torch.zeros(L.ha_hh_counters(), dtype=torch.int32, device="cuda")
    tau = torch.empty(nb, device="cuda")

    def panel(buf, lda, col):
        S = torch.zeros((nb + 1, slen), dtype=torch.float64, device="cuda")
        K.check(L.ha_hh_colsums(K._ptr(buf), 0, m, lda, 0, col, nb, col, K._ptr(S[0]), K._ptr(hpart), K._ptr(hcnt),
                                st), "colsums")
        for j in range(nb):
            last = j + 1 == nb
            K.check(L.ha_hh_step(K._ptr(buf), 0, m, lda, 0, 0, col, nb, j, K._ptr(S[j]),
                                 K._ptr(None) if last else K._ptr(S[j + 1]), K._ptr(tau), K._ptr(None),
                                 K._ptr(hpart), K._ptr(hcnt), st), "step")

    A0 = A.clone()
    t_strided = timed(lambda: panel(A, n, 0))
    P = A0[:, :nb].contiguous()
    t_compact = timed(lambda: panel(P, nb, 0))
    t_copy = timed(lambda: P.copy_(A0[:, :nb]))
    print(json.dumps({"piece": "panel32", "m": m, "strided_ms": t_strided, "compact_ms": t_compact,
                      "copy_in_ms": t_copy}), flush=True)
    del A0, P
    V = torch.randn(m, 256, device="cuda") * 1e-3
    X = torch.randn(256, n - 256, device="cuda")
    C = A[:, 256:]
    flops = 2.0 * m * 256 * (n - 256)
    t_f32 = timed(lambda: K.gemm_f32(V, X, out=C, accumulate=True, alpha=-1.0))
    t_blas = timed(lambda: C.addmm_(V, X, alpha=-1.0))
    t_vtc = timed(lambda: K.vtc64(V, C))
    print(json.dumps({"piece": "update_k256", "m": m, "N": n - 256, "gemm_f32t_ms": t_f32,
                      "gemm_f32t_tf": flops / t_f32 / 1e9, "hipblaslt_ms": t_blas,
                      "hipblaslt_tf": flops / t_blas / 1e9, "vtc64_ms": t_vtc, "vtc64_tf": flops / t_vtc / 1e9}),
          flush=True)
    Cc = torch.empty((m, n - 256), device="cuda")
    Cc.copy_(C)
    t_f32c = timed(lambda: K.gemm_f32(V, X, out=Cc, accumulate=True, alpha=-1.0))
    t_vtcc = timed(lambda: K.vtc64(V, Cc))
    Vi = V[:, :32].contiguous()
    Xi = X[:32, :224].contiguous()
    Ci = A[:, 32:256]
    fi = 2.0 * m * 32 * 224
    ti_f32 = timed(lambda: K.gemm_f32(Vi, Xi, out=Ci, accumulate=True, alpha=-1.0))
    ti_blas = timed(lambda: Ci.addmm_(Vi, Xi, alpha=-1.0))
    ti_vtc = timed(lambda: K._vtc(Vi, Ci, True, st))
    print(json.dumps({"piece": "inner_k32_n224", "gemm_f32t_ms": ti_f32, "hipblaslt_ms": ti_blas,
                      "hh_vtc_ms": ti_vtc, "gemm_f32t_tf": fi / ti_f32 / 1e9}), flush=True)
    print(json.dumps({"piece": "update_k256_contig", "gemm_f32t_ms": t_f32c, "gemm_f32t_tf": flops / t_f32c / 1e9,
                      "vtc64_ms": t_vtcc, "vtc64_tf": flops / t_vtcc / 1e9}), flush=True)


if __name__ == "__main__":
    main()
