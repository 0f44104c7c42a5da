"""
statistical_moments benchmark (reference ``benchmarks/statistical_moments/heat-gpu.py:20-28``):
wall-clock of ``ht.mean`` and ``ht.std`` for axis in {None, 0, 1}.

Default shape: 1e9 float32 per GPU as (rows x 1000), split 0 (BASELINE.json: 1e9-element
float32). Reports GB/s of input read (one pass per call).
"""
import argparse

from benchmarks import common  # noqa: F401
from benchmarks.common import ht, report, setup, timed


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows-per-gpu", type=int, default=1_000_000)
    p.add_argument("--cols", type=int, default=1000)
    p.add_argument("--trials", type=int, default=10)
    a = p.parse_args()
    dev = setup()
    n = a.rows_per_gpu * ht.MPI_WORLD.size
    ht.random.seed(4)
    data = ht.random.rand(n, a.cols, split=0, device=dev)
    for fname, fn in (("mean", ht.mean), ("std", ht.std)):
        for axis in (None, 0, 1):
            t = timed(lambda: fn(data, axis=axis), a.trials)
            report("statistical_moments", {"function": fname, "axis": axis, "shape": [n, a.cols]}, t,
                   {"GB_per_s": 4.0 * n * a.cols / 1e9})


if __name__ == "__main__":
    main()
