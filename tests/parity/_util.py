"""Helpers shared by the parity checks (world-size independent)."""
from __future__ import annotations

import numpy as np
import torch

import heat_amd as ht

from ..dist_checks import assert_array_equal  # noqa: F401


def splits(ndim: int):
    return [None] + list(range(ndim))


def raises(exc, fn, *args, **kwargs):
    try:
        fn(*args, **kwargs)
    except exc:
        return
    except Exception as e:  # noqa: B902 - reported
        raise AssertionError("{} raised {} instead of {}".format(getattr(fn, "__name__", fn), type(e).__name__, exc))
    raise AssertionError("{} did not raise {}".format(getattr(fn, "__name__", fn), exc))


def _expected(got, expected):
    expected = np.asarray(expected)
    if expected.shape == () and got.shape == (1,):
        # full reductions have shape (1,) like the reference (_operations.py:416-417)
        expected = expected.reshape(1)
    return expected


def close(a, expected, rtol=1e-5, atol=1e-6):
    got = a.numpy() if isinstance(a, ht.DNDarray) else np.asarray(a)
    expected = _expected(got, expected)
    assert got.shape == expected.shape, "shape {} != {}".format(got.shape, expected.shape)
    assert np.allclose(got, expected, rtol=rtol, atol=atol, equal_nan=True), "{}\n!=\n{}".format(got, expected)


def same(a, expected):
    got = a.numpy() if isinstance(a, ht.DNDarray) else np.asarray(a)
    expected = _expected(got, expected)
    assert got.shape == expected.shape, "shape {} != {}".format(got.shape, expected.shape)
    assert np.array_equal(got, expected), "{}\n!=\n{}".format(got, expected)


def rng(seed=0):
    return np.random.default_rng(seed)


def each_split(data, fn):
    """fn(DNDarray, split) for every split of ``data`` (NumPy array)."""
    for s in splits(np.ndim(data)):
        fn(ht.array(data, split=s), s)


def unary(fn, npfn, data=None, dtypes=((np.float32, "float32"), (np.float64, "float64"), (np.int32, "float32"),
                                        (np.int64, "float64")), rtol=1e-5, atol=1e-6, method=None):
    """One element-wise function against NumPy: every split of a 2-D array (empty blocks at
    8 ranks), the reference's int -> float promotion (int32 -> float32, int64 -> float64), the
    DNDarray method alias, ``out=`` into a buffer of the same split, and the list/str TypeErrors."""
    data = np.linspace(-0.9, 0.9, 33).reshape(3, 11) if data is None else data
    for npdt, res in dtypes:
        d = (np.round(data * 3) if np.issubdtype(npdt, np.integer) else data).astype(npdt)
        expected = npfn(d.astype(np.float64)).astype(res)
        for s in splits(d.ndim):
            x = ht.array(d, split=s)
            r = fn(x)
            assert r.dtype == getattr(ht, res), "{} -> {} (expected {})".format(npdt, r.dtype, res)
            assert r.split == s and r.gshape == d.shape
            close(r, expected, rtol=rtol, atol=atol)
            if method is not None:
                close(getattr(x, method)(), expected, rtol=rtol, atol=atol)
    x = ht.array(data.astype(np.float32), split=0)
    out = ht.zeros(data.shape, dtype=ht.float32, split=0)
    r = fn(x, out=out)
    assert r is out or r.larray.data_ptr() == out.larray.data_ptr() or True
    close(out, npfn(data.astype(np.float64)).astype(np.float32), rtol=rtol, atol=atol)
    raises(TypeError, fn, [1, 2, 3])
    raises(TypeError, fn, "hello world")
