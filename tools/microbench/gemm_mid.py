"""The LDS-DMA 128-tile GEMM (csrc/gemm_mid.hip: gemm_f32m) against the register-staged 128-tile
kernel (gemm_f32s), the 256-tile kernel (gemm_f32t) and hipBLASLt (torch.mm at precision "highest"),
one process: square products below the north-star size with a K-slice scan per kernel, and the
Householder trailing-update shape C[m, N] -= V[m, 256] X[256, N] (C a column slice of a row-major
[m, 4096] matrix). One JSON line per shape: best time per kernel and its slice count.
Env GM_SHAPES=sq|upd|all (default all), GM_ROWS (update rows, default 1.25e6)."""
import json
import os
import time

import torch

from heat_amd.ops import kernels as K


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def best(fn, slices, reps):
    res = {}
    for s in slices:
        try:
            res[s] = timed(lambda: fn(s), reps)
        except Exception as e:  # noqa: BLE001 - a slice count a kernel refuses
            res[s] = float("inf")
            print(json.dumps({"error": str(e), "slices": s}), flush=True)
    s = min(res, key=res.get)
    return res[s], s


def main():
    torch.manual_seed(0)
    torch.set_float32_matmul_precision("highest")
    which = os.environ.get("GM_SHAPES", "all")
    if which in ("sq", "all"):
        for n in (1024, 2048, 3072, 4096, 6144):
            a = torch.randn(n, n, device="cuda")
            b = torch.randn(n, n, device="cuda")
            reps = 50 if n <= 2048 else 10
            ref = a.double() @ b.double()
            c = K.gemm_f32_small(a, b, kernel="mid256")
            err = float((c.double() - ref).abs().max())
            t_lib = timed(lambda: torch.mm(a, b), reps)
            sl = (1, 2, 3, 4, 6, 8, 12) if n <= 3072 else (1, 2, 3)
            t_m, s_m = best(lambda s: K.gemm_f32_small(a, b, slices=s, kernel="mid128"), sl, reps)
            t_w, s_w = best(lambda s: K.gemm_f32_small(a, b, slices=s, kernel="mid256"), sl, reps)
            t_6, s_6 = best(lambda s: K.gemm_f32_small(a, b, slices=s, kernel="mid64"), sl[:4], reps)
            t_x, s_x = best(lambda s: K.gemm_f32_small(a, b, slices=s, kernel="mid128x64"), sl[:4], reps)
            t_g, s_g = best(lambda s: K.gemm_f32_small(a, b, slices=s, kernel="mid128g2"), sl, reps)
            t_s, s_s = best(lambda s: K.gemm_f32_small(a, b, slices=s, kernel="s"), sl, reps)
            t_t, s_t = best(lambda s: K.gemm_f32(a, b, slices=s), sl, reps)
            from heat_amd.core.linalg import basics
            t_p = timed(lambda: basics.fgemm(a, b), reps)   # what ht.matmul runs (the plan's pick)
            plan = basics._native_plan(n, n, n)
            fl = 2.0 * n ** 3
            print(json.dumps({"M": n, "N": n, "K": n, "hipblaslt_ms": round(t_lib, 4), "f32m_ms": round(t_m, 4),
                              "f32m_slices": s_m, "f32m256_ms": round(t_w, 4), "f32m256_slices": s_w,
                              "f32m256_vs_lib": round(t_w / t_lib, 3), "f32m64_ms": round(t_6, 4), "f32m64_slices": s_6,
                              "f32m64_vs_lib": round(t_6 / t_lib, 3), "f32m128x64_ms": round(t_x, 4),
                              "f32m128x64_slices": s_x, "f32m128x64_vs_lib": round(t_x / t_lib, 3),
                              "f32m128g2_ms": round(t_g, 4), "f32m128g2_slices": s_g,
                              "f32m128g2_vs_lib": round(t_g / t_lib, 3), "f32m128g2_vs_f32m": round(t_g / t_m, 3),
                              "f32s_ms": round(t_s, 4), "f32s_slices": s_s,
                              "f32t_ms": round(t_t, 4), "f32t_slices": s_t, "f32m_vs_lib": round(t_m / t_lib, 3),
                              "f32s_vs_lib": round(t_s / t_lib, 3), "plan": list(plan), "plan_ms": round(t_p, 4),
                              "plan_vs_lib": round(t_p / t_lib, 3), "hipblaslt_tf": round(fl / t_lib / 1e9, 1),
                              "f32m_tf": round(fl / t_m / 1e9, 1), "f32m_max_abs_err": err}), flush=True)
            del a, b, ref, c
            torch.cuda.empty_cache()
    if which in ("upd", "all"):
        m = int(float(os.environ.get("GM_ROWS", "1250000")))
        A = torch.randn(m, 4096, device="cuda")
        for N, Kd in ((3840, 256), (2048, 256), (768, 256), (3840, 512)):
            C = A[:, 4096 - N:]
            V = torch.randn(m, Kd, device="cuda")
            X = torch.randn(Kd, N, device="cuda") * 1e-3
            rows = slice(0, 4096)
            ref = C[rows].double() - V[rows].double() @ X.double()
            K.gemm_f32_small(V, X, out=C, accumulate=True, alpha=-1.0, kernel="mid256")
            err = float((C[rows].double() - ref).abs().max())
            t_lib = timed(lambda: K._exact_addmm_(C, V, X, -1.0), 5)
            t_m = timed(lambda: K.gemm_f32_small(V, X, out=C, accumulate=True, alpha=-1.0, kernel="mid128"), 5)
            t_w = timed(lambda: K.gemm_f32_small(V, X, out=C, accumulate=True, alpha=-1.0, kernel="mid256"), 5)
            t_6 = timed(lambda: K.gemm_f32_small(V, X, out=C, accumulate=True, alpha=-1.0, kernel="mid64"), 5)
            t_x = timed(lambda: K.gemm_f32_small(V, X, out=C, accumulate=True, alpha=-1.0, kernel="mid128x64"), 5)
            t_g = timed(lambda: K.gemm_f32_small(V, X, out=C, accumulate=True, alpha=-1.0, kernel="mid128g2"), 5)
            t_s = timed(lambda: K.gemm_f32_small(V, X, out=C, accumulate=True, alpha=-1.0, kernel="s"), 5)
            t_t = timed(lambda: K.gemm_f32(V, X, out=C, accumulate=True, alpha=-1.0), 5)
            fl = 2.0 * m * N * Kd
            print(json.dumps({"M": m, "N": N, "K": Kd, "update": True, "hipblaslt_ms": round(t_lib, 3),
                              "f32m_ms": round(t_m, 3), "f32m256_ms": round(t_w, 3),
                              "f32m256_vs_lib": round(t_w / t_lib, 3), "f32m64_ms": round(t_6, 3),
                              "f32m64_vs_lib": round(t_6 / t_lib, 3), "f32m128x64_ms": round(t_x, 3),
                              "f32m128x64_vs_lib": round(t_x / t_lib, 3), "f32m128g2_ms": round(t_g, 3),
                              "f32m128g2_vs_lib": round(t_g / t_lib, 3), "f32m128g2_vs_f32m": round(t_g / t_m, 3),
                              "f32s_ms": round(t_s, 3), "f32t_ms": round(t_t, 3),
                              "f32m_vs_lib": round(t_m / t_lib, 3), "hipblaslt_tf": round(fl / t_lib / 1e9, 1),
                              "f32m_tf": round(fl / t_m / 1e9, 1), "f32m_max_abs_err_4096rows": err}), flush=True)
            del V, X, ref
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
