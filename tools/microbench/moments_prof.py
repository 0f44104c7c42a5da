"""Whole-call timing of ht.mean / ht.var / ht.std on 1e9 fp32 (1e6 x 1000, one GPU) per axis, for
rocprofv3 --kernel-trace --stats (one fused moments kernel per call expected) and wall clock
(torch.cuda events around 20 calls). JSON lines: ms per call and input TB/s."""
import json

import torch

import heat_amd as ht


def main():
    ht.use_device("gpu")
    ht.random.seed(4)
    x = ht.random.rand(1_000_000, 1000, split=0)
    for name, fn in (("mean", ht.mean), ("var", ht.var), ("std", ht.std)):
        for axis in (None, 0, 1):
            for _ in range(3):
                fn(x, axis=axis)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                r = fn(x, axis=axis)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / 20
            print(json.dumps({"function": name, "axis": axis, "ms": round(ms, 4), "TB_per_s": round(4e9 / ms / 1e9, 3),
                              "out_shape": list(r.shape)}), flush=True)


if __name__ == "__main__":
    main()
