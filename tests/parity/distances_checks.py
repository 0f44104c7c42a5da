"""Parity with ``heat/spatial/tests/test_distances.py``: cdist / rbf / manhattan for every split
combination of X and Y (with and without the quadratic expansion), output splits, values against
SciPy, and the reference's NotImplementedErrors (split-1 operands, >2-D input)."""
import math

import numpy as np
from scipy.spatial.distance import cdist as sp_cdist

import heat_amd as ht

from ._util import close, raises, rng


def test_cdist():
    n = ht.MPI_WORLD.size
    X = ht.ones((n * 2, 4), dtype=ht.float32)
    Y = ht.zeros((n * 2, 4), dtype=ht.float32)
    for q in (False, True):
        d = ht.spatial.cdist(X, quadratic_expansion=q)
        assert d.split is None
        close(d, np.zeros((2 * n, 2 * n)), atol=1e-5)
        d = ht.spatial.rbf(X, quadratic_expansion=q)
        close(d, np.ones((2 * n, 2 * n)), atol=1e-5)
        d = ht.spatial.cdist(X, Y, quadratic_expansion=q)
        close(d, np.full((2 * n, 2 * n), 2.0), atol=1e-5)
    close(ht.spatial.rbf(X, Y, sigma=math.sqrt(2.0)), np.full((2 * n, 2 * n), math.exp(-1.0)), atol=1e-6)
    for e in (False, True):
        close(ht.spatial.manhattan(X, expand=e), np.zeros((2 * n, 2 * n)))
        close(ht.spatial.manhattan(X, Y, expand=e), np.full((2 * n, 2 * n), 4.0))
    a, b = rng(1).standard_normal((13, 5)), rng(2).standard_normal((9, 5))
    for sx in (None, 0):
        for sy in (None, 0):
            x, y = ht.array(a, split=sx), ht.array(b, split=sy)
            for q in (False, True):
                d = ht.spatial.cdist(x, y, quadratic_expansion=q)
                close(d, sp_cdist(a, b), rtol=1e-6, atol=1e-6)
                # reference split rules: X split 0 -> 0; X replicated, Y split 0 -> 1; else None
                assert d.split == (0 if sx == 0 else (1 if sy == 0 else None)), (sx, sy, d.split)
            close(ht.spatial.manhattan(x, y), sp_cdist(a, b, "cityblock"), rtol=1e-9)
            close(ht.spatial.rbf(x, y, sigma=1.5), np.exp(-sp_cdist(a, b) ** 2 / (2 * 1.5 ** 2)), rtol=1e-6)
        close(ht.spatial.cdist(ht.array(a, split=sx)), sp_cdist(a, a), atol=1e-6)
    af = a.astype(np.float32)
    # fp32 quadratic expansion: |x|^2 + |y|^2 - 2xy cancels to ~eps |x|^2 on the diagonal (sqrt -> ~1e-3)
    close(ht.spatial.cdist(ht.array(af, split=0), quadratic_expansion=True), sp_cdist(af, af), atol=2e-3)
    X1 = ht.ones((n * 2, 4), dtype=ht.float32, split=1)
    raises(NotImplementedError, ht.spatial.cdist, X1)
    raises(NotImplementedError, ht.spatial.cdist, X1, Y, quadratic_expansion=False)
    raises(NotImplementedError, ht.spatial.cdist, X, ht.zeros((n * 2, 4), split=1), quadratic_expansion=False)
    Z = ht.ones((n * 2, 6, 3), dtype=ht.float32)
    raises(NotImplementedError, ht.spatial.cdist, Z, quadratic_expansion=False)
    raises(NotImplementedError, ht.spatial.cdist, X, Z, quadratic_expansion=False)
