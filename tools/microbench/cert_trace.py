"""Re-check fraction of the certified assignment along a Lloyd run on the bench.py data
(1.25e7 x 64 standard normal, k = 1024, random init): per step, the fraction of points the
one-term filter could not certify and the certified vs full assignment times."""
import json

import torch

import heat_amd as ht
from heat_amd import ops


def timed(fn):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    r = fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e), r


def main():
    ht.use_device("gpu")
    ht.random.seed(1234)
    x = ht.random.randn(12_500_000, 64, split=0)
    km = ht.cluster.KMeans(n_clusters=1024, init="random", max_iter=1, tol=None, random_state=42)
    km.step(x)
    X = x.larray
    P = ops.kmeans_pack_points(X)
    for it in range(25):
        C = km.cluster_centers_.larray
        tc, (lc, _) = timed(lambda: ops.kmeans_assign(X, C, want_mind=False, packed=P, certified=True))
        frac = int(ops.kmeans_assign.last_rechecked.item()) / X.shape[0]
        tf, (lf, _) = timed(lambda: ops.kmeans_assign(X, C, want_mind=False, packed=P, certified=False))
        print(json.dumps({"step": it, "recheck_frac": round(frac, 4), "certified_ms": round(tc, 3),
                          "full_ms": round(tf, 3), "labels_equal": bool(torch.equal(lc, lf))}), flush=True)
        km.step(x)


if __name__ == "__main__":
    main()
