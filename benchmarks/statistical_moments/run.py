"""
statistical_moments benchmark (reference ``benchmarks/statistical_moments/heat-gpu.py:20-28``):
wall-clock of ``ht.mean`` and ``ht.std`` for axis in {None, 0, 1}.

Default shape: 1e9 float32 per GPU as (rows x 1000), split 0 (BASELINE.json: 1e9-element
float32). Reports GB/s of input read (one pass per call).

Same-node comparator (world of one): the reference's ``torch-gpu.py:20-27``, ``torch.mean`` /
``torch.std`` with the same axis on the same data (``reference_torch_s`` / ``speedup``).
"""
import argparse

from benchmarks import common  # noqa: F401
from benchmarks.common import ht, report, setup, timed, torch_reference


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows-per-gpu", type=int, default=1_000_000)
    p.add_argument("--cols", type=int, default=1000)
    p.add_argument("--trials", type=int, default=10)
    p.add_argument("--no-reference", action="store_true", help="skip the torch comparator")
    a = p.parse_args()
    import torch

    dev = setup()
    n = a.rows_per_gpu * ht.MPI_WORLD.size
    ht.random.seed(4)
    data = ht.random.rand(n, a.cols, split=0, device=dev)
    local = data.larray
    for (fname, fn), tfn in zip((("mean", ht.mean), ("std", ht.std)), (torch.mean, torch.std)):
        for axis in (None, 0, 1):
            t = timed(lambda: fn(data, axis=axis), a.trials)
            ref = None if a.no_reference else torch_reference(lambda: tfn(local, dim=axis), a.trials)  # noqa: B023
            report("statistical_moments", {"function": fname, "axis": axis, "shape": [n, a.cols]}, t,
                   {"GB_per_s": 4.0 * n * a.cols / 1e9}, reference=ref)


if __name__ == "__main__":
    main()
