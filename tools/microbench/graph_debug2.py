"""Which captured part goes wrong on the SECOND replay? (certified assignment off)"""
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
    km.step(x)
    km._certify, km._cert_probe = False, None
    torch.cuda.synchronize()
    C = km.cluster_centers_.larray.clone()
    packed = km._packed(X)
    rec = {}
    lab_e, _ = ops.kmeans_assign(X, C, want_mind=False, packed=packed)
    g, (lab_g, _) = cap(lambda: ops.kmeans_assign(X, C, want_mind=False, packed=packed))
    for r in range(3):
        g.replay()
        torch.cuda.synchronize()
        rec["assign_mismatch_replay%d" % r] = int((lab_g != lab_e).sum())
    s_e, c_e = ops.kmeans_update(X, lab_e, k)
    g2, (s_g, c_g) = cap(lambda: ops.kmeans_update(X, lab_e, k))
    for r in range(3):
        g2.replay()
        torch.cuda.synchronize()
        rec["update_sum_maxdiff_replay%d" % r] = float((s_g - s_e).abs().max())
        rec["update_cnt_maxdiff_replay%d" % r] = float((c_g - c_e).abs().max())
    pk = torch.cat([s_e.reshape(-1).double(), c_e.double()])
    nc_e, sh_e = ops.kmeans_finalize(pk, C)
    g3, (nc_g, sh_g) = cap(lambda: ops.kmeans_finalize(pk, C))
    for r in range(3):
        g3.replay()
        torch.cuda.synchronize()
        rec["finalize_maxdiff_replay%d" % r] = float((nc_g - nc_e).abs().max())
        rec["finalize_shift_replay%d" % r] = [float(sh_g), float(sh_e)]
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
