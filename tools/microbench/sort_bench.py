"""Native radix sort (ops.sort_rows) vs torch.sort(stable=True) on the device; JSON lines."""
import json
import time

import torch

from heat_amd import ops


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for shape in [(12_500_000,), (100_000_000,), (1000, 12_500), (64, 1_000_000)]:
    for dt in (torch.float32, torch.int32):
        x = torch.randn(shape, device="cuda") if dt == torch.float32 else \
            torch.randint(-2**30, 2**30, shape, device="cuda", dtype=torch.int32)
        a = timed(lambda: ops.sort_rows(x))
        b = timed(lambda: torch.sort(x, dim=-1, stable=True))
        v, i = ops.sort_rows(x)
        rv, ri = torch.sort(x, dim=-1, stable=True)
        print(json.dumps({"shape": shape, "dtype": str(dt), "radix_ms": round(a, 3), "torch_sort_ms": round(b, 3),
                          "equal": bool(torch.equal(v, rv) and torch.equal(i, ri))}), flush=True)
