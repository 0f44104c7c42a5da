"""Which part of the k-means step misbehaves under HIP graph capture? Captures the assign and the
update separately and compares each with eager results."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import heat_amd as ht  # noqa: E402
from heat_amd import ops  # noqa: E402


def cap(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    return g, out


def main():
    ht.use_device("gpu")
    ht.random.seed(1234)
    n, k, f = 2_000_000, 1024, 64
    x = ht.random.randn(n, f, split=0)
    X = x.larray
    km = ht.cluster.KMeans(n_clusters=k, init="random", max_iter=1, tol=None, random_state=42)
    for _ in range(4):
        km.step(x)
    torch.cuda.synchronize()
    C = km.cluster_centers_.larray.clone()
    rec = {"certify_flag": bool(km._certify)}
    packed = km._packed(X)
    lab_e, _ = ops.kmeans_assign(X, C, want_mind=False, packed=packed)
    g, (lab_g, _) = cap(lambda: ops.kmeans_assign(X, C, want_mind=False, packed=packed))
    g.replay()
    torch.cuda.synchronize()
    rec["assign_label_mismatch"] = int((lab_g != lab_e).sum())
    s_e, c_e = ops.kmeans_update(X, lab_e, k)
    g2, (s_g, c_g) = cap(lambda: ops.kmeans_update(X, lab_e, k))
    g2.replay()
    torch.cuda.synchronize()
    rec["update_sum_maxdiff"] = float((s_g - s_e).abs().max())
    rec["update_count_maxdiff"] = float((c_g - c_e).abs().max())
    newc_e, _ = km._centroid_step(X, C, x.comm, False)
    g3, (newc_g, _) = cap(lambda: km._centroid_step(X, C, x.comm, False))
    g3.replay()
    torch.cuda.synchronize()
    rec["step_maxdiff"] = float((newc_g - newc_e).abs().max())
    # replay twice more: does a second replay still agree?
    g3.replay()
    torch.cuda.synchronize()
    rec["step_maxdiff_replay2"] = float((newc_g - newc_e).abs().max())
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
