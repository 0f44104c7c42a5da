"""Probe: fp16-in / fp32-out GEMM throughput through torch.mm(out_dtype=float32) (hipBLASLt) vs
fp32 GEMM, on the shapes a K-concatenated fp16x3 split GEMM would use."""
import torch

dev = torch.device("cuda", 0)


def t(fn, it=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


for (m, k, n) in [(65536, 4096, 4096), (87381, 4096, 4096), (4096, 65536, 4096)]:
    a = torch.randn(m, k, device=dev)
    b = torch.randn(k, n, device=dev)
    ms32 = t(lambda: torch.mm(a, b))
    a3 = torch.randn(m, 3 * k, device=dev).half()
    b3 = torch.randn(3 * k, n, device=dev).half()
    ms16 = t(lambda: torch.mm(a3, b3, out_dtype=torch.float32))
    b3t = b3.t().contiguous().t()
    ms16t = t(lambda: torch.mm(a3, b3t, out_dtype=torch.float32))
    a3t = a3.t().contiguous().t()
    ms16tt = t(lambda: torch.mm(a3t, b3, out_dtype=torch.float32))
    ms16h = t(lambda: torch.mm(a3, b3))
    f = 2.0 * m * n * k
    print(f"m={m} k={k} n={n}: fp32 {ms32:.2f} ms ({f / ms32 / 1e9:.0f} TF), f16x3(K=3k)->f32 NN {ms16:.2f} ms "
          f"(eff {f / ms16 / 1e9:.0f} TF, raw {3 * f / ms16 / 1e9:.0f} TF), NT {ms16t:.2f} ms, TN {ms16tt:.2f} ms, "
          f"fp16 out {ms16h:.2f} ms", flush=True)
    del a, b, a3, b3, b3t, a3t
