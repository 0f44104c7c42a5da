"""
Tall-skinny linear algebra (BASELINE.json: TSQR / matmul 1e7 x 4096 split 0 on 8 GPUs):
``ht.linalg.qr`` (TSQR, R only and Q+R) and ``ht.matmul`` (A @ B with B replicated, and the Gram
matrix A^T A which contracts over the split axis: local GEMM + one all-reduce).
"""
import argparse

from benchmarks import common  # noqa: F401
from benchmarks.common import ht, report, setup, timed


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows-per-gpu", type=int, default=1_250_000)
    p.add_argument("--cols", type=int, default=4096)
    p.add_argument("--trials", type=int, default=3)
    p.add_argument("--ops", default="matmul,gram,qr_r,qr")
    p.add_argument("--precision", default="highest", choices=["highest", "high"],
                   help="torch float32 matmul precision: 'high' runs the fp16x3 split GEMM")
    a = p.parse_args()
    import torch

    torch.set_float32_matmul_precision(a.precision)
    dev = setup()
    m, n = a.rows_per_gpu * ht.MPI_WORLD.size, a.cols
    ht.random.seed(5)
    A = ht.random.randn(m, n, split=0, device=dev)
    ops = a.ops.split(",")
    if "matmul" in ops:
        B = ht.random.randn(n, n, device=dev)
        t = timed(lambda: ht.matmul(A, B), a.trials)
        report("linalg", {"op": "matmul A@B", "m": m, "n": n, "precision": a.precision}, t, {"gflops": 2.0 * m * n * n / 1e9})
        del B
    if "gram" in ops:
        t = timed(lambda: ht.matmul(A.T, A), a.trials)
        report("linalg", {"op": "gram A^T A", "m": m, "n": n, "precision": a.precision}, t, {"gflops": 2.0 * m * n * n / 1e9})
    if "qr_r" in ops:
        t = timed(lambda: ht.linalg.qr(A, calc_q=False), a.trials)
        report("linalg", {"op": "tsqr R", "m": m, "n": n, "precision": a.precision}, t, {"gflops": (2.0 * m * n * n - 2.0 * n ** 3 / 3) / 1e9})
    if "qr" in ops:
        t = timed(lambda: ht.linalg.qr(A), a.trials)
        report("linalg", {"op": "tsqr Q,R", "m": m, "n": n, "precision": a.precision}, t, {"gflops": (4.0 * m * n * n - 4.0 * n ** 3 / 3) / 1e9})


if __name__ == "__main__":
    main()
