"""Parity with ``heat/core/tests/test_exponential.py``: every function against NumPy on every split,
the int -> float promotion rules, the method aliases, ``out=`` buffers and the TypeErrors."""
import numpy as np

import heat_amd as ht

from ._util import close, raises, same, splits, unary

POS = np.linspace(0.05, 3.0, 33).reshape(3, 11)
GT1 = np.linspace(1.0, 4.0, 33).reshape(3, 11)


def test_exp():
    unary(ht.exp, np.exp, method="exp")


def test_expm1():
    unary(ht.expm1, np.expm1, method="expm1")


def test_exp2():
    unary(ht.exp2, np.exp2, method="exp2")


def test_log():
    unary(ht.log, np.log, data=POS, method="log")


def test_log2():
    unary(ht.log2, np.log2, data=POS, method="log2")


def test_log10():
    unary(ht.log10, np.log10, data=POS, method="log10")


def test_log1p():
    unary(ht.log1p, np.log1p, data=POS, method="log1p")


def test_sqrt():
    unary(ht.sqrt, np.sqrt, data=POS, method="sqrt")


def test_square():
    unary(ht.square, np.square, method="square")


def _binary_exp(fn, npfn):
    a = np.linspace(-3, 3, 24).reshape(4, 6)
    b = np.linspace(2, -1, 24).reshape(4, 6)
    for s in splits(2):
        for dt, res in ((np.float32, ht.float32), (np.float64, ht.float64)):
            r = fn(ht.array(a.astype(dt), split=s), ht.array(b.astype(dt), split=s))
            assert r.dtype == res and r.split == s
            close(r, npfn(a, b), rtol=1e-5)
        close(fn(ht.array(a, split=s), ht.array(b[0], split=None)), npfn(a, b[0]))
    raises(TypeError, fn, [1, 2, 3], [1, 2, 3])
    raises(TypeError, fn, "hello world", "hello world")


def test_logaddexp():
    _binary_exp(ht.logaddexp, np.logaddexp)


def test_logaddexp2():
    _binary_exp(ht.logaddexp2, np.logaddexp2)


def test_sqrt_method():
    for dt, res in ((ht.float32, ht.float32), (ht.float64, ht.float64), (ht.int32, ht.float32), (ht.int64, ht.float64)):
        for s in (None, 0):
            r = ht.arange(25, dtype=dt, split=s).sqrt()
            assert r.dtype == res and r.split == s
            close(r, np.sqrt(np.arange(25.0)))


def test_sqrt_out_of_place():
    n = ht.arange(30, dtype=ht.float32)
    for s in (None, 1):
        out = ht.zeros((3, 30), dtype=ht.float32, split=s)
        r = ht.sqrt(ht.array(np.broadcast_to(np.arange(30.0, dtype=np.float32), (3, 30)).copy(), split=s), out=out)
        assert r.dtype == ht.float32 and r.gshape == (3, 30)
        close(out, np.broadcast_to(np.sqrt(np.arange(30.0)), (3, 30)))
    r = ht.sqrt(n, out=ht.zeros(30, dtype=ht.float32))
    assert float(n.sum(axis=0).item()) == 435 and n.gshape == (30,)
    raises(TypeError, ht.sqrt, n, "hello world")
