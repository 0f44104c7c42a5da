"""Does the memory-bound k-means update overlap with the MFMA-bound assignment? One Lloyd step's
assign + update on 12.5M x 64 points, k = 1024: sequential vs the points cut into P slabs, slab
p's update (side stream) running under slab p+1's assignment (main stream). JSON lines."""
import json

import torch

import heat_amd as ht
from heat_amd.ops import kernels as K


def timed(fn, reps=10):
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
    n, f, k = 12_500_000, 64, 1024
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn(n, f, device="cuda", generator=g)
    C = X[torch.randperm(n, device="cuda", generator=g)[:k]].clone()
    packed = K.kmeans_pack_points(X)

    def seq():
        lab, _ = K.kmeans_assign(X, C, want_mind=False, packed=packed)
        return K.kmeans_update(X, lab, k)

    ref_s, ref_c = seq()
    print(json.dumps({"mode": "sequential", "ms": round(timed(seq), 4)}), flush=True)
    side = torch.cuda.Stream()

    def piped(P):
        main = torch.cuda.current_stream()
        bounds = [(n * p // P) // 256 * 256 for p in range(P)] + [n]
        parts = []
        for p in range(P):
            a, b = bounds[p], bounds[p + 1]
            pk = K.PackedPoints(packed.planes[a:b], packed.sx[a:b], b - a, f, packed.key)
            lab, _ = K.kmeans_assign(X[a:b], C, want_mind=False, packed=pk)
            ev = torch.cuda.Event()
            ev.record(main)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                parts.append(K.kmeans_update(X[a:b], lab, k))
                lab.record_stream(side)
        main.wait_stream(side)
        sums = torch.stack([s for s, _ in parts]).sum(0)
        counts = torch.stack([c for _, c in parts]).sum(0)
        return sums, counts

    for P in (2, 4, 8):
        s, c = piped(P)
        err = float(((s - ref_s).abs().max() / ref_s.abs().max()))
        ok = bool(torch.equal(c, ref_c))
        print(json.dumps({"mode": "pipelined", "P": P, "ms": round(timed(lambda: piped(P)), 4), "sum_rel_err": err,
                          "counts_equal": ok}), flush=True)


if __name__ == "__main__":
    main()
