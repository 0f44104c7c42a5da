"""Parity with ``heat/core/tests/test_trigonometrics.py``: every function against NumPy on every split,
the int -> float promotion rules, the method aliases, ``out=`` buffers and the TypeErrors."""
import numpy as np

import heat_amd as ht

from ._util import close, raises, same, splits, unary

POS = np.linspace(0.05, 3.0, 33).reshape(3, 11)
GT1 = np.linspace(1.0, 4.0, 33).reshape(3, 11)


def test_arccos():
    unary(ht.arccos, np.arccos)


def test_acosh():
    unary(ht.acosh, np.arccosh, data=GT1)


def test_arcsin():
    unary(ht.arcsin, np.arcsin)


def test_asinh():
    unary(ht.asinh, np.arcsinh)


def test_arctan():
    unary(ht.arctan, np.arctan)


def test_atanh():
    unary(ht.atanh, np.arctanh)


def test_degrees():
    unary(ht.degrees, np.degrees)


def test_deg2rad():
    unary(ht.deg2rad, np.deg2rad)


def test_cos():
    unary(ht.cos, np.cos)


def test_cosh():
    unary(ht.cosh, np.cosh)


def test_rad2deg():
    unary(ht.rad2deg, np.rad2deg)


def test_radians():
    unary(ht.radians, np.radians)


def test_sin():
    unary(ht.sin, np.sin)


def test_sinh():
    unary(ht.sinh, np.sinh)


def test_tan():
    unary(ht.tan, np.tan)


def test_tanh():
    unary(ht.tanh, np.tanh)


def test_arctan2():
    y = np.array([-1.0, -1.0, 1.0, 1.0, 0.0, 2.0, -3.0, 0.5])
    x = np.array([-1.0, 1.0, 1.0, -1.0, -2.0, 0.0, 4.0, 0.5])
    for s in (None, 0):
        for dt, res in ((np.float32, ht.float32), (np.float64, ht.float64), (np.int32, ht.float32),
                        (np.int64, ht.float64)):
            r = ht.arctan2(ht.array(y.astype(dt), split=s), ht.array(x.astype(dt), split=s))
            assert r.dtype == res and r.split == s, (dt, r.dtype)
            close(r, np.arctan2(y.astype(dt).astype(np.float64), x.astype(dt).astype(np.float64)), rtol=1e-5)
    close(ht.arctan2(ht.array(y, split=0), 1.0), np.arctan2(y, 1.0))
    raises(TypeError, ht.arctan2, [1, 2], [3, 4])
