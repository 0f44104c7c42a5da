"""Split-K scan of the hand-written fp32 GEMMs against hipBLASLt (exact fp32): for each shape the
256-tile kernel (gemm_f32t) at K-slice counts 1..16 and the 128-tile kernel (gemm_f32s) at 1..16,
to derive the routing rule of ht.matmul's local products. One JSON line per shape."""
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
    shapes = [(1024, 1024, 1024), (2048, 2048, 2048), (3072, 3072, 3072), (4096, 4096, 4096), (6144, 6144, 6144),
              (8192, 8192, 8192), (2048, 2048, 65536), (65536, 512, 512), (100000, 256, 256), (1250000, 3840, 256),
              (4096, 4096, 1024), (16384, 1024, 4096)]
    for M, N, Kd in shapes:
        a = torch.randn(M, Kd, device="cuda")
        b = torch.randn(Kd, N, device="cuda")
        rec = {"M": M, "N": N, "K": Kd, "lib_ms": round(timed(lambda: torch.mm(a, b)), 4)}
        for s in (1, 2, 3, 4, 6, 8, 12, 16):
            if Kd // s < 64 or (s > 1 and s * M * N * 4 > (4 << 30)):
                continue
            rec["f32t_s%d" % s] = round(timed(lambda: K.gemm_f32(a, b, slices=s)), 4)
            rec["f32s_s%d" % s] = round(timed(lambda: K.gemm_f32_small(a, b, slices=s)), 4)
        best = min((v, k) for k, v in rec.items() if k.startswith("f32"))
        rec["best"], rec["best_vs_lib"] = best[1], round(best[0] / rec["lib_ms"], 3)
        print(json.dumps(rec), flush=True)
        del a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
