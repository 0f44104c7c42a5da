"""
kmeans benchmark (reference ``benchmarks/kmeans/heat-gpu.py:22-28``): wall-clock of
``KMeans(n_clusters, max_iter).fit(data)`` with init="random".

* ``--case reference``: the reference protocol, k=8, 30 iterations (tol disabled so every run does
  all 30), data ``--rows`` x ``--features`` per GPU (weak scaling; default 1.25e7 x 64).
* ``--case northstar``: BASELINE.json config, k=1024 on 1.25e7 x 64 per GPU (1e8 x 64 on 8 GPUs);
  reports per-iteration time and GFLOP/s of the distance computation (2 n k f per iteration).

Same-node comparator (world of one): the reference's ``torch-gpu.py:9-55`` algorithm in plain torch
on the same data - ``torch.cdist`` to the centroids, ``argmin``, then one masked sum per cluster.
For ``reference`` all iterations are timed; for ``northstar`` (1024 masked passes per iteration)
one iteration is timed and the record's ``reference_torch_s`` is scaled to ``iterations``.
"""
import argparse

from benchmarks import common  # noqa: F401
from benchmarks.common import ht, report, setup, timed, torch_reference


def torch_kmeans(x, k: int, iters: int, seed: int = 0):
    """The reference's torch comparator (``benchmarks/kmeans/torch-gpu.py``): random init from a
    permutation, ``torch.cdist`` + ``argmin`` assignment, one masked pass per cluster for the new
    centroids, squared centroid shift per iteration (no convergence test: tol = -1)."""
    import torch

    g = torch.Generator(device="cpu").manual_seed(seed)
    cent = x[torch.randperm(x.shape[0], generator=g)[:k].to(x.device)]
    new = cent.clone()
    for _ in range(iters):
        match = torch.cdist(x, cent).argmin(dim=1, keepdim=True)
        for i in range(k):
            sel = (match == i).to(torch.int64)
            pts = (x * sel).sum(dim=0, keepdim=True)
            cnt = sel.sum(dim=0, keepdim=True).clamp(1, torch.iinfo(torch.int64).max)
            new[i: i + 1, :] = pts / cnt
        shift = ((cent - new) ** 2).sum()
        cent = new.clone()
    return cent, shift


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--case", default="northstar", choices=["reference", "northstar"])
    p.add_argument("--rows-per-gpu", type=int, default=12_500_000)
    p.add_argument("--features", type=int, default=64)
    p.add_argument("--clusters", type=int, default=None)
    p.add_argument("--iterations", type=int, default=None)
    p.add_argument("--trials", type=int, default=3)
    p.add_argument("--precision", default="fast", choices=["fast", "exact"])
    p.add_argument("--no-reference", action="store_true", help="skip the torch comparator")
    a = p.parse_args()
    dev = setup()
    k = a.clusters or (8 if a.case == "reference" else 1024)
    iters = a.iterations or (30 if a.case == "reference" else 10)
    n = a.rows_per_gpu * ht.MPI_WORLD.size
    ht.random.seed(2)
    data = ht.random.randn(n, a.features, split=0, device=dev)

    def fit():
        km = ht.cluster.KMeans(n_clusters=k, init="random", max_iter=iters, tol=None, random_state=5)
        km.precision = a.precision
        km.fit(data)

    t = timed(fit, a.trials)
    ref = None
    if not a.no_reference:
        local = data.larray
        if a.case == "reference":
            ref = torch_reference(lambda: torch_kmeans(local, k, iters), a.trials)
        else:   # one iteration of 1024 masked passes, scaled to the fit's iteration count
            ref = [s * iters for s in torch_reference(lambda: torch_kmeans(local, k, 1), 1, warmup=0)]
    report("kmeans", {"case": a.case, "n": n, "f": a.features, "k": k, "iterations": iters,
                      "precision": a.precision}, t,
           {"gflops": 2.0 * n * k * a.features * iters / 1e9, "iterations_per_s": iters}, reference=ref)


if __name__ == "__main__":
    main()
