"""Parity with ``heat/core/tests/test_indexing.py``: nonzero and where (one- and three-argument)
on every split against NumPy, result splits and dtypes, use of the result as an index, and the
errors."""
import numpy as np

import heat_amd as ht

from ._util import raises, rng, same, splits

A = np.array([[1, 2, 3], [4, 5, 6], [7, 8, 9]])


def test_nonzero():
    for s in splits(2):
        a = ht.array([[1, 2, 3], [4, 5, 2], [7, 8, 9]], split=s)
        nz = ht.nonzero(a > 3)
        assert nz.gshape == (5, 2) and nz.dtype == ht.int64
        assert nz.split == (None if s is None else 0)
        same(nz, np.argwhere(np.array([[1, 2, 3], [4, 5, 2], [7, 8, 9]]) > 3))
    a = ht.array(A, split=1)
    nz = (a > 3).nonzero()
    assert nz.gshape == (6, 2) and nz.split == 0
    a[nz] = 10.0
    assert bool(ht.all(a[nz] == 10).item())
    x = rng(1).standard_normal((7, 3, 5))
    for s in splits(3):
        same(ht.nonzero(ht.array(x, split=s) > 0.5), np.argwhere(x > 0.5))
    v = rng(2).integers(0, 3, 17)
    for s in (None, 0):
        same(ht.nonzero(ht.array(v, split=s)), np.flatnonzero(v))


def test_where():
    for s in splits(2):
        a = ht.array(A, split=s)
        wh = ht.where(a > 3)
        assert wh.gshape == (6, 2) and wh.dtype == ht.int64 and wh.split == (None if s is None else 0)
        same(wh, np.argwhere(A > 3))
    f = np.array([[0.0, 1.0, 2.0], [0.0, 2.0, 4.0], [0.0, 3.0, 6.0]], dtype=np.float32)
    for s in splits(2):
        a = ht.array(f, split=s)
        wh = ht.where(a < 4.0, a, -1)
        assert wh.gshape == (3, 3) and wh.dtype == ht.float32 and wh.split == s
        same(wh, np.where(f < 4.0, f, -1).astype(np.float32))
        assert bool(ht.all(wh[ht.nonzero(a >= 4)] == -1).item())
        same(a[ht.nonzero(a < 4)], f[f < 4].astype(np.float32))
        same(ht.where(a < 4.0, -1.0, a), np.where(f < 4.0, -1.0, f).astype(np.float32))
        same(ht.where(a < 4.0, a, ht.array(f * 10, split=s)), np.where(f < 4.0, f, f * 10).astype(np.float32))
    x = rng(3).standard_normal((9, 4))
    y = rng(4).standard_normal((9, 4))
    for s in splits(2):
        same(ht.where(ht.array(x, split=s) > 0, ht.array(x, split=s), ht.array(y, split=s)), np.where(x > 0, x, y))
    cond = ht.array(A) > 3
    raises(TypeError, ht.where, cond, ht.array(f))
    # the reference raises NotImplementedError for operands split along different axes; here they
    # are aligned with one all-to-all (documented in core/_operations.py)
    same(ht.where(cond, ht.ones((3, 3), split=0), ht.zeros((3, 3), split=1)), np.where(A > 3, 1.0, 0.0).astype(np.float32))
