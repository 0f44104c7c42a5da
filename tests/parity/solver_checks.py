"""Parity with ``heat/core/linalg/tests/test_solver.py``: conjugate gradients on a distributed
diagonal and a dense SPD system, and its TypeError/RuntimeErrors; plus Lanczos."""
import numpy as np

import heat_amd as ht

from ._util import close, raises, rng


def test_cg():
    size = ht.MPI_WORLD.size * 3
    b = ht.arange(1, size + 1, dtype=ht.float32, split=0)
    A = ht.manipulations.diag(b)
    x0 = ht.random.rand(size, dtype=b.dtype, split=b.split)
    res = ht.linalg.cg(A, b, x0)
    assert ht.allclose(ht.ones(b.shape, dtype=b.dtype, split=b.split), res, atol=1e-3)
    M = rng(1).standard_normal((12, 12))
    S = M @ M.T + 12 * np.eye(12)
    rhs = rng(2).standard_normal(12)
    for s in (None, 0):
        x = ht.linalg.cg(ht.array(S, split=s), ht.array(rhs, split=s), ht.zeros(12, dtype=ht.float64, split=s))
        close(x, np.linalg.solve(S, rhs), rtol=1e-6, atol=1e-6)
    raises(TypeError, ht.linalg.cg, A, np.arange(1, size + 1), x0)
    raises(RuntimeError, ht.linalg.cg, A, A, x0)
    raises(RuntimeError, ht.linalg.cg, b, b, x0)
    raises(RuntimeError, ht.linalg.cg, A, b, A)


def test_lanczos():
    M = rng(3).standard_normal((30, 30))
    S = (M + M.T) / 2
    for s in (None, 0):
        V, T = ht.linalg.lanczos(ht.array(S, split=s), m=30)
        ev = np.sort(np.linalg.eigvalsh(T.numpy()))
        close(ev, np.sort(np.linalg.eigvalsh(S)), rtol=1e-6, atol=1e-6)
        Vn = V.numpy()
        close(Vn.T @ Vn, np.eye(30), atol=1e-6)
