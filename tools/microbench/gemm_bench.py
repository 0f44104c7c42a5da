"""Exact fp32 GEMM: heat_amd MFMA kernel vs torch.mm (hipBLASLt) on the linalg north-star shape
(a 1.25e6 x 4096 row block @ 4096 x 4096, the per-GPU slice of 1e7 x 4096 on 8 GPUs) and squares.
Interleaved rounds in one process; prints JSON lines (ms, TFLOP/s)."""
import json
import sys

import torch

from heat_amd import ops


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


def main():
    shapes = [(8192, 8192, 8192), (4096, 4096, 4096), (1_250_000, 4096, 4096)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]]
    for m, k, n in shapes:
        a = torch.randn(m, k, device="cuda")
        b = torch.randn(k, n, device="cuda")
        c = torch.empty(m, n, device="cuda")
        reps = 3 if m * n * k > 1e12 else 10
        fl = 2.0 * m * n * k
        res = {"shape": [m, k, n]}
        from heat_amd.ops import kernels as K

        best = {}
        for rnd in range(2):
            for bk in (2, 4):
                K._GEMM_BK = bk
                t = timeit(lambda: ops.gemm_f32(a, b, out=c), reps)
                best["nt%d" % bk] = min(best.get("nt%d" % bk, 1e30), t)
            t = timeit(lambda: torch.mm(a, b, out=c), reps)
            best["blas"] = min(best.get("blas", 1e30), t)
            t = timeit(lambda: ops.gemm_h3(a, b, out=c), reps)
            best["h3_fused"] = min(best.get("h3_fused", 1e30), t)
            t = timeit(lambda: ops.gemm_f16x3(a, b, out=c), reps)
            best["h3_blas_tripled"] = min(best.get("h3_blas_tripled", 1e30), t)
        for key, t in best.items():
            res[key + "_ms"] = t
            res[key + "_tflops"] = fl / (t * 1e-3) / 1e12
        print(json.dumps(res), flush=True)
        del a, b, c
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
