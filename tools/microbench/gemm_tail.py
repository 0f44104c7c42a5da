"""Wave-quantisation tail of the 128-tile gemm_f32m at 6144^3 (2304 tiles = 4.5 rounds of 512
workgroup slots): the whole product in one launch vs the first M1 rows in one launch plus the
remaining rows split over K (their slices summed by ha_sum_slices32), hipBLASLt alongside.
One JSON line per (M1, tail slices)."""
import json
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
    torch.set_float32_matmul_precision("highest")
    for n in (6144, 5120, 7168):
        a = torch.randn(n, n, device="cuda")
        b = torch.randn(n, n, device="cuda")
        c = torch.empty(n, n, device="cuda")
        ref = a.double() @ b.double()
        t_lib = timed(lambda: torch.mm(a, b))
        t_one = timed(lambda: K.gemm_f32_small(a, b, out=c, slices=1, kernel="mid128"))
        print(json.dumps({"n": n, "hipblaslt_ms": round(t_lib, 4), "one_launch_ms": round(t_one, 4),
                          "one_vs_lib": round(t_one / t_lib, 3)}), flush=True)
        for m1 in range(n // 2, n, 512):
            for ts in (2, 3):
                def run():
                    K.gemm_f32_small(a[:m1], b, out=c[:m1], slices=1, kernel="mid128")
                    K.gemm_f32_small(a[m1:], b, out=c[m1:], slices=ts, kernel="mid128")
                t = timed(run)
                err = float((c.double() - ref).abs().max())
                print(json.dumps({"n": n, "m1": m1, "tail_slices": ts, "ms": round(t, 4), "vs_lib": round(t / t_lib, 3),
                                  "vs_one": round(t / t_one, 3), "max_abs_err": err}), flush=True)
        del a, b, c, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
