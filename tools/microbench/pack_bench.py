"""Native one-pass block pack (csrc/pack.hip) vs narrow().contiguous() + torch.cat for the send
buffer of a split 0 -> split 1 resplit on 8 ranks (a 1e9-byte-class slab)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from heat_amd import ops


def bench(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    out = []
    for shape, axis in (((16384, 8192), 1), ((8192, 64, 512), 1), ((125_000_000 // 8,), 0)):
        t = torch.randn(shape, device="cuda")
        p = 8
        n = shape[axis]
        counts = [n // p + (1 if r < n % p else 0) for r in range(p)]
        off = [sum(counts[:r]) for r in range(p)]
        nat = bench(lambda: ops.pack_blocks(t, axis, counts))
        ref = bench(lambda: torch.cat([t.narrow(axis, off[r], counts[r]).reshape(-1) for r in range(p)]))
        flat = ops.pack_blocks(t, axis, counts)
        unp = bench(lambda: ops.unpack_blocks(flat, t.shape, axis, counts))
        gb = 2 * t.numel() * 4 / 1e9
        rec = {"shape": list(shape), "axis": axis, "blocks": p, "native_pack_ms": round(nat, 4),
               "torch_narrow_cat_ms": round(ref, 4), "native_unpack_ms": round(unp, 4),
               "native_pack_TBps": round(gb / nat, 2), "torch_TBps": round(gb / ref, 2)}
        print(json.dumps(rec), flush=True)
        out.append(rec)


if __name__ == "__main__":
    main()
