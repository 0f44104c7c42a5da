"""Parity with ``heat/core/tests/test_logical.py``: all/any over every axis and split (shape (1,)
for a full reduction, bool dtype, ``out=``), allclose/isclose (scalars, mixed splits), the IEEE
predicates and the element-wise logical operators."""
import numpy as np
import torch

import heat_amd as ht

from ._util import close, raises, rng, same, splits

V = np.array([[0.0, 1.0, 2.0, -1.0], [3.0, 0.0, np.inf, 1.0], [1.0, 1.0, 1.0, 1.0]])


def _reduce_check(fn, npfn):
    for data in (np.ones(9), np.ones((3, 3, 3)), (rng(1).random((5, 3, 4)) > 0.3).astype(np.float32),
                 np.arange(-4, 5)):
        for s in splits(data.ndim):
            x = ht.array(data, split=s)
            r = fn(x)
            assert r.shape == (1,) and r.dtype == ht.bool and r.split is None and r.larray.dtype == torch.bool
            assert bool(r.item()) == bool(npfn(data))
            out = ht.zeros((1,))
            fn(x, out=out)
            assert float(out.item()) == float(npfn(data))
            for ax in range(data.ndim):
                r = fn(x, axis=ax)
                assert r.dtype == ht.bool and r.split == (None if s in (None, ax) else (s if s < ax else s - 1))
                same(r, npfn(data, axis=ax))
                same(fn(x, axis=ax, keepdim=True), npfn(data, axis=ax, keepdims=True))
            if data.ndim == 3:
                same(fn(x, axis=(0, 1)), npfn(data, axis=(0, 1)))
                out = ht.zeros(data.shape[1:])
                fn(x, axis=0, out=out)
                same(out, npfn(data, axis=0).astype(np.float32))
    raises(ValueError, fn, ht.ones(9), axis=1)
    raises(ValueError, fn, ht.ones(9), axis=-2)
    raises(ValueError, fn, ht.ones((4, 4)), axis=0, out=ht.zeros((1,)))
    raises(TypeError, fn, ht.ones(9), axis="bad_axis_type")


def test_all():
    _reduce_check(ht.all, np.all)
    assert bool(ht.ones((3, 3), split=0).all().item())


def test_any():
    _reduce_check(ht.any, np.any)
    assert not bool(ht.zeros((3, 3), split=1).any().item())


def test_allclose():
    size = ht.MPI_WORLD.size
    a = ht.float32([[2, 2], [2, 2]])
    b = ht.float32([[2.00005, 2.00005], [2.00005, 2.00005]])
    c = ht.zeros((4 * size, 6), split=0)
    d = ht.zeros((4 * size, 6), split=1)
    e = ht.zeros((4 * size, 6))
    assert not ht.allclose(a, b)
    assert ht.allclose(a, b, atol=1e-4) and ht.allclose(a, b, rtol=1e-4)
    assert ht.allclose(a, 2) and ht.allclose(a, 2.0) and ht.allclose(2, a)
    assert ht.allclose(c, d) and ht.allclose(c, e) and e.allclose(c)
    x = rng(2).standard_normal((7, 5))
    for s in splits(2):
        assert ht.allclose(ht.array(x, split=s), ht.array(x + 1e-9, split=s))
        assert not ht.allclose(ht.array(x, split=s), ht.array(x + 1e-3, split=s))
    n = np.array([1.0, np.nan])
    assert not ht.allclose(ht.array(n), ht.array(n))
    assert ht.allclose(ht.array(n), ht.array(n), equal_nan=True)
    raises(TypeError, ht.allclose, a, (2, 2, 2, 2))
    raises(TypeError, ht.allclose, a, "?")
    raises(TypeError, ht.allclose, "?", a)


def test_isclose():
    size = ht.MPI_WORLD.size
    a = ht.float32([[2, 2], [2, 2]])
    b = ht.float32([[2.00005, 2.00005], [2.00005, 2.00005]])
    c = ht.zeros((4 * size, 6), split=0)
    d = ht.zeros((4 * size, 6), split=1)
    e = ht.zeros((4 * size, 6))
    assert ht.isclose(a, b).shape == (2, 2)
    assert not ht.isclose(a, b)[0][0].item()
    assert ht.isclose(a, b, atol=1e-04)[0][1].item() and ht.isclose(a, b, rtol=1e-04)[1][0].item()
    assert ht.isclose(a, 2)[0][1].item() and ht.isclose(a, 2.0)[0][0].item() and ht.isclose(2, a)[1][1].item()
    assert ht.isclose(c, d).shape == (4 * size, 6)
    assert ht.isclose(c, e)[0][0].item() and e.isclose(c)[-1][-1].item()
    assert isinstance(ht.isclose(2.0, 2.00005), bool)
    x = rng(3).standard_normal((6, 4))
    y = x + rng(4).standard_normal((6, 4)) * 1e-6
    for s in splits(2):
        same(ht.isclose(ht.array(x, split=s), ht.array(y, split=s), rtol=1e-6, atol=1e-7),
             np.isclose(x, y, rtol=1e-6, atol=1e-7))
    raises(TypeError, ht.isclose, a, (2, 2, 2, 2))
    raises(TypeError, ht.isclose, a, "?")
    raises(TypeError, ht.isclose, "?", a)


def _pred(fn, npfn):
    data = np.array([1.0, np.inf, -np.inf, np.nan, -0.0, 3.5, -2.0])
    for s in (None, 0):
        r = fn(ht.array(data, split=s))
        assert r.dtype == ht.bool and r.split == s
        same(r, npfn(data))
    for dt in (ht.bool, ht.int32, ht.int64, ht.float32):
        for s in splits(2):
            r = fn(ht.ones((6, 5), dtype=dt, split=s))
            assert r.dtype == ht.bool and r.split == s
            same(r, npfn(np.ones((6, 5))))


def test_isfinite():
    _pred(ht.isfinite, np.isfinite)


def test_isinf():
    _pred(ht.isinf, np.isinf)


def test_isnan():
    _pred(ht.isnan, np.isnan)


def test_isneginf():
    _pred(ht.isneginf, np.isneginf)
    out = ht.empty(7, dtype=ht.bool)
    ht.isneginf(ht.array([1.0, np.inf, -np.inf, np.nan, -0.0, 3.5, -2.0]), out=out)
    same(out, [False, False, True, False, False, False, False])


def test_isposinf():
    _pred(ht.isposinf, np.isposinf)
    out = ht.empty(7, dtype=ht.bool)
    ht.isposinf(ht.array([1.0, np.inf, -np.inf, np.nan, -0.0, 3.5, -2.0]), out=out)
    same(out, [False, True, False, False, False, False, False])


def _logical_bin(fn, npfn):
    a = np.array([[True, False], [True, True], [False, False]])
    b = np.array([[True, True], [False, True], [True, False]])
    for s in splits(2):
        r = fn(ht.array(a, split=s), ht.array(b, split=s))
        assert r.dtype == ht.bool and r.split == s
        same(r, npfn(a, b))
        same(fn(ht.array(a.astype(np.float32), split=s), ht.array(b.astype(np.int64), split=s)), npfn(a, b))
        same(fn(ht.array(a, split=s), True), npfn(a, True))


def test_logical_and():
    _logical_bin(ht.logical_and, np.logical_and)


def test_logical_or():
    _logical_bin(ht.logical_or, np.logical_or)


def test_logical_xor():
    _logical_bin(ht.logical_xor, np.logical_xor)


def test_logical_not():
    a = np.array([[True, False], [0.0, 2.0], [False, True]])
    for s in splits(2):
        r = ht.logical_not(ht.array(a, split=s))
        assert r.dtype == ht.bool and r.split == s
        same(r, np.logical_not(a))
    out = ht.empty((3, 2), dtype=ht.bool)
    ht.logical_not(ht.array(a), out=out)
    same(out, np.logical_not(a))


def test_signbit():
    data = np.array([-1.0, -0.0, 0.0, 2.0, -np.inf, np.inf, -3.5])
    for s in (None, 0):
        r = ht.signbit(ht.array(data, split=s))
        assert r.dtype == ht.bool and r.split == s
        same(r, np.signbit(data))
    same(ht.signbit(ht.array([-1, 0, 3], dtype=ht.int32)), [True, False, False])
    out = ht.empty(7, dtype=ht.bool)
    ht.signbit(ht.array(data), out=out)
    same(out, np.signbit(data))
