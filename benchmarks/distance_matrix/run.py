"""
distance_matrix benchmark (reference ``benchmarks/distance_matrix/heat-gpu.py:20-34``): wall-clock
of ``cdist(data, data, quadratic_expansion=False/True)``.

* ``--case susy``: the reference's strong-scaling size, 40k rows x 18 features (SUSY), full
  matrix materialised (6.4 GB), split 0.
* ``--case northstar``: BASELINE.json config, 1e6 x 128 vs itself; the 4 TB result is streamed
  tile by tile (``ht.spatial.cdist_stream``) through one reused HBM tile.
* ``--case knn``: the northstar size reduced to every row's ``--k`` nearest rows by the fused
  distance + top-k kernel (``ht.spatial.cdist_topk``; no matrix at all).
GFLOP/s convention: 3*m*n*f for the exact path (sub, mul, add), 2*m*n*f for the expansion GEMM.

Same-node comparator (world of one, ``--case susy``): the reference's ``torch-gpu.py:20-25``,
``torch.cdist(data, data)`` on the same data - ``reference_torch_s`` / ``speedup`` in each record.
"""
import argparse

from benchmarks import common  # noqa: F401  (sets sys.path)
from benchmarks.common import ht, report, setup, timed, torch_reference


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--case", default="susy", choices=["susy", "northstar", "knn"])
    p.add_argument("--rows", type=int, default=None)
    p.add_argument("--features", type=int, default=None)
    p.add_argument("--trials", type=int, default=5)
    p.add_argument("--k", type=int, default=8, help="knn: neighbours per row")
    p.add_argument("--no-reference", action="store_true", help="skip the torch comparator")
    a = p.parse_args()
    dev = setup()
    n = a.rows or (40_000 if a.case == "susy" else 1_000_000)
    f = a.features or (18 if a.case == "susy" else 128)
    ht.random.seed(1)
    data = ht.random.rand(n, f, split=0, device=dev)
    if a.case == "knn":
        t = timed(lambda: ht.spatial.cdist_topk(data, data, a.k), a.trials)
        report("distance_matrix", {"case": "knn", "n": n, "f": f, "k": a.k}, t,
               {"gflops": 2.0 * n * n * f / 1e9, "distances_per_s": float(n) * n})
        return
    ref = None
    if a.case == "susy" and not a.no_reference:
        import torch

        local = data.larray
        ref = torch_reference(lambda: torch.cdist(local, local), a.trials)   # reference torch-gpu.py:23
    for qe in (False, True):
        if a.case == "susy":
            fn = lambda: ht.spatial.cdist(data, data, quadratic_expansion=qe)  # noqa: E731
        else:
            fn = lambda: ht.spatial.cdist_stream(data, data, lambda d, i, j: None,  # noqa: E731
                                                 quadratic_expansion=qe)
        t = timed(fn, a.trials)
        report("distance_matrix", {"case": a.case, "n": n, "f": f, "quadratic_expansion": qe}, t,
               {"gflops": (2.0 if qe else 3.0) * n * n * f / 1e9, "distances_per_s": float(n) * n}, reference=ref)
        if a.case == "susy":
            # Y = None (the reference's symmetric path): each distance pair computed once
            t = timed(lambda: ht.spatial.cdist(data, quadratic_expansion=qe), a.trials)  # noqa: B023
            report("distance_matrix", {"case": a.case, "n": n, "f": f, "quadratic_expansion": qe, "Y": None}, t,
                   {"gflops": (2.0 if qe else 3.0) * n * n * f / 1e9, "distances_per_s": float(n) * n},
                   reference=ref)


if __name__ == "__main__":
    main()
