"""Parity with ``heat/core/tests/test_rounding.py``: abs/fabs, ceil/floor/trunc/round, clip and
modf against NumPy on every split, dtype rules (``dtype=`` casts, fabs -> float), ``out=``
buffers (tuples for modf) and the TypeErrors/ValueErrors."""
import numpy as np
import torch

import heat_amd as ht

from ._util import close, raises, rng, same, splits

D = np.array([[-5.7, -2.5, -0.5, 0.0], [0.49, 0.5, 1.5, 2.5], [3.2, -3.8, 7.0, -0.01]])


def test_abs():
    x = ht.arange(-10, 10, dtype=ht.float32, split=0)
    r = ht.abs(x)
    assert r.dtype == ht.float32 and float(r.sum(axis=0).item()) == 100
    for dt in (ht.int8, ht.int16, ht.int32, ht.int64):
        f = ht.fabs(ht.arange(-10.5, 10.5, dtype=dt, split=0))
        assert f.dtype in (ht.float32, ht.float64) and float(f.sum(axis=0).item()) == 100.0
    for dt in (ht.float32, ht.float64):
        f = ht.fabs(ht.arange(-10.5, 10.5, dtype=dt, split=0))
        assert f.dtype == dt and float(f.sum(axis=0).item()) == 110.5
    out = ht.zeros(20, split=0)
    ht.absolute(x, out=out)
    assert float(out.sum(axis=0).item()) == 100
    out = ht.zeros(21, split=0)
    ht.fabs(ht.arange(-10.5, 10.5, dtype=ht.float32, split=0), out=out)
    assert float(out.sum(axis=0).item()) == 110.5
    r = ht.abs(ht.arange(-10, 10, dtype=ht.int64), dtype=ht.float32)
    assert r.dtype == ht.float32 and r.larray.dtype == torch.float32 and float(r.sum().item()) == 100
    for s in splits(2):
        same(ht.abs(ht.array(D, split=s)), np.abs(D))
        same(ht.array(D, split=s).abs(), np.abs(D))
        same(abs(ht.array(D, split=s)), np.abs(D))
    raises(TypeError, ht.absolute, "hello")
    raises(TypeError, ht.array(D).abs, out=1)
    raises(TypeError, ht.array(D).absolute, out=ht.array(D), dtype=3.2)
    raises(TypeError, ht.fabs, "hello")
    raises(TypeError, ht.array(D).fabs, out=1)


def _rounder(fn, npfn, method):
    for dt in (np.float32, np.float64):
        d = D.astype(dt)
        for s in splits(2):
            r = fn(ht.array(d, split=s))
            assert r.dtype == (ht.float32 if dt == np.float32 else ht.float64) and r.split == s
            same(r, npfn(d))
            same(getattr(ht.array(d, split=s), method)(), npfn(d))
    out = ht.zeros(D.shape, split=0)
    fn(ht.array(D.astype(np.float32), split=0), out=out)
    same(out, npfn(D.astype(np.float32)))
    raises(TypeError, fn, [0, 1, 2, 3])
    raises(TypeError, fn, object())


def test_ceil():
    _rounder(ht.ceil, np.ceil, "ceil")


def test_floor():
    _rounder(ht.floor, np.floor, "floor")


def test_trunc():
    _rounder(ht.trunc, np.trunc, "trunc")


def test_round():
    _rounder(ht.round, np.round, "round")
    x = rng(1).standard_normal((5, 7)) * 100
    for s in splits(2):
        for dec in (0, 1, 2, -1):
            close(ht.round(ht.array(x, split=s), dec), np.round(x, dec), rtol=1e-9, atol=1e-9)
        r = ht.array(x, split=s, dtype=ht.float64).round(dtype=ht.float32)
        assert r.dtype == ht.float32
        same(r, np.round(x).astype(np.float32))
    f = ht.array(D, dtype=ht.float32)
    raises(TypeError, ht.round, f, 1, 1)
    raises(TypeError, ht.round, f, dtype=np.int_)


def test_clip():
    x = ht.arange(20, dtype=ht.float32, split=0)
    c = x.clip(5, 15)
    assert c.dtype == ht.float32 and float(c.sum(axis=0).item()) == 195
    c = ht.arange(20, dtype=ht.int64, split=0).clip(4, 16)
    assert c.dtype == ht.int64 and int(c.sum(axis=0).item()) == 194
    for s in splits(2):
        same(ht.clip(ht.array(D, split=s), -1.0, 2.0), np.clip(D, -1.0, 2.0))
        same(ht.clip(ht.array(D, split=s), None, 0.5), np.clip(D, None, 0.5))
        same(ht.clip(ht.array(D, split=s), -0.5, None), np.clip(D, -0.5, None))
    out = ht.empty(20, dtype=ht.float32, split=0)
    ht.clip(x, 5, 15, out=out)
    same(out, np.clip(np.arange(20.0), 5, 15))
    raises(TypeError, ht.clip, torch.arange(10), 2, 5)
    raises(ValueError, ht.arange(20).clip, None, None)
    raises(TypeError, ht.clip, ht.arange(20), 5, 15, out=torch.arange(20))


def test_modf():
    size = ht.MPI_WORLD.size
    step = 10.0 / (2 * size)
    for dt in (np.float32, np.float64):
        a = np.arange(-5.0, 5.0, step, dtype=dt)
        frac, whole = np.modf(a)
        for s in (None, 0):
            f, w = ht.array(a, split=s).modf()
            assert f.dtype == w.dtype == (ht.float32 if dt == np.float32 else ht.float64)
            assert f.split == w.split == s
            same(f, frac)
            same(w, whole)
            outs = (ht.zeros_like(ht.array(a, split=s)), ht.zeros_like(ht.array(a, split=s)))
            ht.array(a, split=s).modf(out=outs)
            same(outs[0], frac)
            same(outs[1], whole)
    f32 = ht.array(np.arange(4.0, dtype=np.float32))
    f64 = ht.array(np.arange(4.0))
    raises(TypeError, ht.modf, [0, 1, 2, 3])
    raises(TypeError, ht.modf, object())
    raises(TypeError, ht.modf, f32, 1)
    raises(ValueError, ht.modf, f32, (f32, f32, f64))
    raises(TypeError, ht.modf, f32, (f32, 2))
