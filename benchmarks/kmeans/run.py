"""
kmeans benchmark (reference ``benchmarks/kmeans/heat-gpu.py:22-28``): wall-clock of
``KMeans(n_clusters, max_iter).fit(data)`` with init="random".

* ``--case reference``: the reference protocol, k=8, 30 iterations (tol disabled so every run does
  all 30), data ``--rows`` x ``--features`` per GPU (weak scaling; default 1.25e7 x 64).
* ``--case northstar``: BASELINE.json config, k=1024 on 1.25e7 x 64 per GPU (1e8 x 64 on 8 GPUs);
  reports per-iteration time and GFLOP/s of the distance computation (2 n k f per iteration).
"""
import argparse

from benchmarks import common  # noqa: F401
from benchmarks.common import ht, report, setup, timed


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--case", default="northstar", choices=["reference", "northstar"])
    p.add_argument("--rows-per-gpu", type=int, default=12_500_000)
    p.add_argument("--features", type=int, default=64)
    p.add_argument("--clusters", type=int, default=None)
    p.add_argument("--iterations", type=int, default=None)
    p.add_argument("--trials", type=int, default=3)
    p.add_argument("--precision", default="fast", choices=["fast", "exact"])
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
    report("kmeans", {"case": a.case, "n": n, "f": a.features, "k": k, "iterations": iters,
                      "precision": a.precision}, t,
           {"gflops": 2.0 * n * k * a.features * iters / 1e9, "iterations_per_s": iters})


if __name__ == "__main__":
    main()
