"""Parity with ``heat/core/tests/test_relational.py``: the six comparisons against NumPy on every
split, scalar and broadcast operands, bool results, ``ht.equal`` semantics and the errors."""
import numpy as np

import heat_amd as ht

from ._util import raises, rng, same, splits

A = np.array([[1.0, 2.0], [3.0, 4.0]])
B = np.array([[2.0, 2.0], [2.0, 2.0]])


def _cmp(fn, npfn, op):
    for s in splits(2):
        a, b = ht.array(A, split=s), ht.array(B, split=s)
        r = fn(a, b)
        assert r.dtype == ht.bool and r.split == s
        same(r, npfn(A, B))
        same(fn(a, 2.0), npfn(A, 2.0))
        same(fn(2.0, a), npfn(2.0, A))
        same(fn(a, ht.array([2.0, 3.0])), npfn(A, np.array([2.0, 3.0])))
        same(op(a, b), npfn(A, B))
        same(op(a, 3), npfn(A, 3))
    x = rng(1).integers(0, 4, (9, 3))
    y = rng(2).integers(0, 4, (9, 3))
    for s in splits(2):
        same(fn(ht.array(x, split=s), ht.array(y.astype(np.float32), split=s)), npfn(x, y.astype(np.float32)))
    raises(ValueError, fn, ht.array(A), ht.array([[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]]))
    raises(TypeError, fn, ht.array(A), ht.array)
    raises(TypeError, fn, "self.a_tensor", "s")


def test_eq():
    _cmp(ht.eq, np.equal, lambda a, b: a == b)


def test_ne():
    _cmp(ht.ne, np.not_equal, lambda a, b: a != b)


def test_ge():
    _cmp(ht.ge, np.greater_equal, lambda a, b: a >= b)


def test_gt():
    _cmp(ht.gt, np.greater, lambda a, b: a > b)


def test_le():
    _cmp(ht.le, np.less_equal, lambda a, b: a <= b)


def test_lt():
    _cmp(ht.lt, np.less, lambda a, b: a < b)


def test_equal():
    for s in splits(2):
        a = ht.array(A, split=s)
        assert ht.equal(a, ht.array(A, split=s)) and ht.equal(a, ht.array(A))
        assert not ht.equal(a, ht.array(B, split=s))
        assert ht.equal(ht.array(B, split=s), 2.0) and not ht.equal(a, 2.0)
        assert not ht.equal(a, ht.array([[1.0, 2.0, 3.0]]))
    x = rng(3).standard_normal((11, 4))
    for s in splits(2):
        y = x.copy()
        y[10, 3] += 1
        assert ht.equal(ht.array(x, split=s), ht.array(x, split=s))
        assert not ht.equal(ht.array(x, split=s), ht.array(y, split=s))
    raises(TypeError, ht.equal, ht.array(A), ht.array)
