"""A/B of the moments kernels on 1e9 fp32 (1e6 x 1000): the row kernel over the flat array with
the fused last-block epilogue vs partials only (out = null), and the column kernel (axis 0) at
several row chunks per CU (HEAT_MOM_COL_CHUNKS_PER_CU). JSON lines, kernel time by CUDA events."""
import ctypes
import json
import os

import torch

import heat_amd as ht
from heat_amd import ops
from heat_amd.ops import kernels as K


def ev_time(fn, reps=20):
    for _ in range(3):
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
    ht.use_device("gpu")
    x = torch.rand(1_000_000, 1000, device="cuda")
    L = ops.lib()
    st = ctypes.c_void_p(ops.stream_ptr(x.device))
    ncu = K.num_cus(x.device)
    numel = x.numel()
    part = torch.empty((4096, 3), dtype=torch.float64, device="cuda")
    for nch in (2048, 4096):
        ms = ev_time(lambda: L.ha_moments_rows(K._ptr(x), 1, numel, numel, nch, K._ptr(part), None, 1, 0.0, None, st))
        print(json.dumps({"kernel": "rows", "nchunks": nch, "fused": False, "ms": round(ms, 4),
                          "TB_per_s": round(4e9 / ms / 1e9, 3)}), flush=True)
    for cpc in (4, 8, 16):
        os.environ["HEAT_MOM_ROW_CHUNKS_PER_CU"] = str(cpc)
        r = K.moments(x, axis=None, final="var")
        err = abs(float(r) - float(x.double().var(correction=0)))
        ms = ev_time(lambda: K.moments(x, axis=None, final="var"))
        print(json.dumps({"kernel": "rows", "chunks_per_cu": cpc, "fused": True, "ms": round(ms, 4),
                          "TB_per_s": round(4e9 / ms / 1e9, 3), "abs_err": err}), flush=True)
    os.environ.pop("HEAT_MOM_ROW_CHUNKS_PER_CU")
    for cpc in (1, 2, 3, 4):
        os.environ["HEAT_MOM_COL_CHUNKS_PER_CU"] = str(cpc)
        r = K.moments(x, axis=0, final="mean")
        err = float((r.double() - x.double().mean(0)).abs().max())
        ms = ev_time(lambda: K.moments(x, axis=0, final="mean"))
        print(json.dumps({"kernel": "cols", "chunks_per_cu": cpc, "ms": round(ms, 4),
                          "TB_per_s": round(4e9 / ms / 1e9, 3), "max_err": err}), flush=True)


if __name__ == "__main__":
    main()
