"""Square and skinny fp32 GEMMs below the north-star size: the hand-written 256 x 256-tile kernels
(exact gemm_f32t, fp16x3 gemm_h3t) and the 128 x 128-tile split-K kernel (gemm_f32s) against hipBLASLt (torch.mm at precision "highest") - where
does a grid of few 256 x 256 tiles leave the 256 CUs idle? One JSON line per shape."""
import json
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


def main():
    torch.manual_seed(0)
    shapes = [(1024, 1024, 1024), (2048, 2048, 2048), (3072, 3072, 3072), (4096, 4096, 4096), (6144, 6144, 6144),
              (8192, 8192, 8192), (2048, 2048, 65536), (65536, 512, 512), (100000, 256, 256), (512, 512, 1000000),
              (1250000, 3840, 256)]
    for M, N, Kd in shapes:
        a = torch.randn(M, Kd, device="cuda")
        b = torch.randn(Kd, N, device="cuda")
        torch.set_float32_matmul_precision("highest")
        t_f32 = timed(lambda: K.gemm_f32(a, b))
        t_lib = timed(lambda: torch.mm(a, b))
        t_h3 = timed(lambda: K.gemm_h3(a, b))
        t_s = timed(lambda: K.gemm_f32_small(a, b))
        fl = 2.0 * M * N * Kd
        tiles = -(-M // 256) * -(-N // 256)
        print(json.dumps({"M": M, "N": N, "K": Kd, "tiles": tiles, "gemm_f32t_ms": round(t_f32, 4),
                          "hipblaslt_ms": round(t_lib, 4), "gemm_h3t_ms": round(t_h3, 4),
                          "gemm_f32t_tf": round(fl / t_f32 / 1e9, 1), "hipblaslt_tf": round(fl / t_lib / 1e9, 1),
                          "gemm_h3t_tf": round(fl / t_h3 / 1e9, 1), "gemm_f32s_ms": round(t_s, 4),
                          "gemm_f32s_tf": round(fl / t_s / 1e9, 1), "f32s_vs_lib": round(t_s / t_lib, 3)}), flush=True)
        del a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
