"""GEMM A/B in one process: the 256-tile kernels (``gemm_tiled.hip``: exact ``gemm_f32t``, fused
fp16x3 ``gemm_h3t``) vs the round-2 128-tile kernels and torch.mm (hipBLASLt: fp32, and the
tripled-K fp16 split of ``ops.gemm_f16x3``) on the linalg north-star shape (a 1.25e6 x 4096 row
block @ 4096 x 4096, the per-GPU slice of 1e7 x 4096 on 8 GPUs), squares and the Gram A^T A.
Interleaved rounds, best of rounds; prints JSON lines (ms, TFLOP/s fp32-equivalent, max error
relative to the fp32-GEMM bound on a row sample)."""
import json
import sys

import torch

from heat_amd import ops
from heat_amd.ops import kernels as K


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def err_ratio(c, a, b, rows):
    ref = a[rows].double() @ b.double()
    bound = a.shape[1] * 2.0 ** -24 * (a[rows].abs().double() @ b.abs().double()) + 1e-30
    return float(((c[rows].double() - ref).abs() / bound).max())


def main():
    shapes = [(8192, 8192, 8192), (4096, 4096, 4096), (1_250_000, 4096, 4096), ("gram", 1_250_000, 4096)]
    rounds = 2
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    if "--quick" in sys.argv:
        rounds = 1
    if args:
        shapes = []
        for s in args:
            if s.startswith("gram"):
                _, m, n = s.split(":")
                shapes.append(("gram", int(m), int(n)))
            else:
                shapes.append(tuple(int(v) for v in s.split("x")))
    torch.manual_seed(0)
    for shp in shapes:
        if shp[0] == "gram":
            _, m, n = shp
            x = torch.randn(m, n, device="cuda")
            a, b = x.t(), x
            M, Kd, N = n, m, n
        else:
            M, Kd, N = shp
            a = torch.randn(M, Kd, device="cuda")
            b = torch.randn(Kd, N, device="cuda")
        c = torch.empty(M, N, device="cuda")
        reps = 2 if M * N * Kd > 1e13 else (3 if M * N * Kd > 1e12 else 10)
        fl = 2.0 * M * N * Kd
        res = {"shape": list(shp)}
        variants = {
            "f32t": lambda: ops.gemm_f32(a, b, out=c),
            "f32_v1": lambda: K.gemm_f32_v1(a, b, out=c),
            "blas_f32": lambda: torch.mm(a, b, out=c),
            "h3t": lambda: ops.gemm_h3(a, b, out=c),
            "h3_v1": lambda: K.gemm_h3_v1(a, b, out=c),
            "blas_f16x3": lambda: ops.gemm_f16x3(a, b, out=c),
        }
        only = [a.split("=", 1)[1].split(",") for a in sys.argv if a.startswith("--only=")]
        if only:
            variants = {k: v for k, v in variants.items() if k in only[0]}
        rows = torch.randint(0, M, (64,), device="cuda")
        best = {}
        for rnd in range(rounds):
            for key, fn in variants.items():
                try:
                    t = timeit(fn, reps)
                except Exception as e:  # noqa: BLE001
                    res[key + "_error"] = str(e)[:200]
                    continue
                best[key] = min(best.get(key, 1e30), t)
                if rnd == 0:
                    res[key + "_err"] = round(err_ratio(c, a, b, rows), 4)
        for key, t in best.items():
            res[key + "_ms"] = round(t, 4)
            res[key + "_tflops"] = round(fl / (t * 1e-3) / 1e12, 2)
        print(json.dumps(res), flush=True)
        del a, b, c
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
