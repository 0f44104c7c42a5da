"""Parity with ``heat/core/tests/test_complex_math.py``: abs/angle/conjugate/imag/real of
complex64/complex128 arrays on every split against NumPy, the real result dtypes, and complex
factories."""
import numpy as np

import heat_amd as ht

from ._util import close, same, splits

C1 = np.array([1.0, 1.0j, 1 + 1j, -2 + 2j, 3 - 3j])
C2 = np.array([[1.0, 1.0j], [1 + 1j, -2 + 2j], [3 - 3j, -4 - 4j]])


def _each(fn, npfn, real_result=True, **kw):
    for data in (C1, C2):
        for cdt, rdt in ((ht.complex64, ht.float32), (ht.complex128, ht.float64)):
            for s in splits(data.ndim):
                a = ht.array(data, split=s, dtype=cdt)
                r = fn(a, **kw)
                assert r.dtype is (rdt if real_result else cdt), (r.dtype, cdt)
                assert r.shape == data.shape and r.split == s
                close(r, npfn(data.astype(np.complex128)), rtol=1e-6, atol=1e-6)


def test_abs():
    _each(ht.absolute, np.abs)
    a = ht.array(C1.tolist())
    assert a.dtype is ht.complex64 and ht.abs(a).dtype is ht.float


def test_angle():
    _each(ht.angle, np.angle)
    _each(ht.angle, lambda z: np.angle(z, deg=True), deg=True)
    r = ht.angle(ht.array([1.0, -1.0, 2.0]))
    close(r, np.angle(np.array([1.0, -1.0, 2.0])))


def test_conjugate():
    _each(ht.conjugate, np.conjugate, real_result=False)
    _each(ht.conj, np.conj, real_result=False)
    a = ht.array(C2, split=0)
    close(a.conj(), np.conj(C2))
    same(ht.conj(ht.array([1.0, -2.0], split=0)), np.array([1.0, -2.0], dtype=np.float32))


def test_imag():
    _each(ht.imag, np.imag)
    same(ht.imag(ht.array([1.0, 2.0])), np.zeros(2, dtype=np.float32))
    close(ht.array(C2, split=1).imag, np.imag(C2))


def test_real():
    _each(ht.real, np.real)
    same(ht.real(ht.array([1.0, 2.0], split=0)), np.array([1.0, 2.0], dtype=np.float32))
    close(ht.array(C2, split=0).real, np.real(C2))


def test_full():
    a = ht.full((4, 4), 1 + 1j)
    assert a.dtype is ht.complex64 and a.shape == (4, 4)
    close(a, np.full((4, 4), 1 + 1j))
    for s in splits(2):
        b = ht.full((5, 3), 2 - 1j, dtype=ht.complex128, split=s)
        assert b.dtype is ht.complex128 and b.split == s
        close(b, np.full((5, 3), 2 - 1j))
    z = ht.zeros((3, 2), dtype=ht.complex64, split=0)
    assert z.dtype is ht.complex64
    same(z, np.zeros((3, 2), dtype=np.complex64))
