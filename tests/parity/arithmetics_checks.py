"""Parity with ``heat/core/tests/test_arithmetics.py``: every arithmetic function over every split,
scalar / array / broadcast operands, dtype promotion and the reference's error cases."""
import operator

import numpy as np
import torch

import heat_amd as ht

from ._util import close, each_split, raises, rng, same, splits

A = np.array([[1.0, 2.0], [3.0, 4.0]], dtype=np.float32)
B = np.full((2, 2), 2.0, dtype=np.float32)
V2 = np.array([2.0, 2.0], dtype=np.float32)
V3 = np.array([2.0, 2.0, 2.0], dtype=np.float32)
I = np.array([[1, 2], [3, 4]], dtype=np.int32)
BOOL1 = np.array([False, True, False, True])
BOOL2 = np.array([False, False, True, True])


def _binary(fn, npfn, a=A, b=B):
    for sa in splits(a.ndim):
        for sb in splits(np.ndim(b)):
            close(fn(ht.array(a, split=sa), ht.array(b, split=sb)), npfn(a, b))
    close(fn(ht.array(a, split=0), 2.0), npfn(a, np.float32(2.0)))
    close(fn(2.0, ht.array(a, split=1)), npfn(np.float32(2.0), a))
    close(fn(ht.array(a, split=0), ht.array(V2)), npfn(a, V2))


def _errors(fn):
    raises(ValueError, fn, ht.array(A), ht.array(V3))
    raises(TypeError, fn, ht.array(A), (2, 2))
    raises(TypeError, fn, "T", "s")


def test_add():
    _binary(ht.add, np.add)
    assert ht.equal(ht.add(2.0, 2.0), ht.float32(4.0))
    _errors(ht.add)


def test_sub():
    _binary(ht.sub, np.subtract)
    _errors(ht.sub)


def test_mul():
    _binary(ht.mul, np.multiply)
    _errors(ht.mul)


def test_div():
    _binary(ht.div, np.divide)
    close(ht.div(ht.array(I), 2), I / 2)
    _errors(ht.div)


def test_pow():
    _binary(ht.pow, np.power)
    close(ht.pow(ht.array(I, split=0), 2), I ** 2)
    _errors(ht.pow)


def test_fmod():
    a = np.array([[-3.5, 2.0], [7.25, -1.0]], dtype=np.float32)
    _binary(ht.fmod, np.fmod, a, B)
    same(ht.fmod(ht.array(np.array([-7, 5, 9]), split=0), 4), np.fmod(np.array([-7, 5, 9]), 4))
    _errors(ht.fmod)


def test_mod():
    a = np.array([[-3.5, 2.0], [7.25, -1.0]], dtype=np.float32)
    _binary(ht.mod, np.mod, a, B)
    same(ht.mod(ht.array(np.array([-7, 5, 9]), split=0), 4), np.mod(np.array([-7, 5, 9]), 4))
    same(ht.remainder(ht.array(np.array([-7, 5, 9])), -4), np.remainder(np.array([-7, 5, 9]), -4))
    _errors(ht.mod)


def _bitwise(fn, npfn):
    iv, iv4 = np.array([2, 2], dtype=np.int32), np.array([2, 2, 2, 2], dtype=np.int32)
    for s in splits(2):
        same(fn(ht.array(I, split=s), 2), npfn(I, 2))
        same(fn(ht.array(I, split=s), ht.array(iv)), npfn(I, iv))
    for s in splits(1):
        same(fn(ht.array(BOOL1, split=s), ht.array(BOOL2, split=s)), npfn(BOOL1, BOOL2))
    raises(TypeError, fn, ht.array(A), ht.array(B))
    raises(ValueError, fn, ht.array(iv), ht.array(iv4))
    raises(TypeError, fn, ht.array(A), (2, 2))
    raises(TypeError, fn, "T", "s")
    raises(TypeError, fn, ht.array(I), "s")
    raises(TypeError, fn, 2, 2.0)


def test_bitwise_and():
    _bitwise(ht.bitwise_and, np.bitwise_and)


def test_bitwise_or():
    _bitwise(ht.bitwise_or, np.bitwise_or)


def test_bitwise_xor():
    _bitwise(ht.bitwise_xor, np.bitwise_xor)


def test_invert():
    for s in splits(2):
        same(ht.invert(ht.array(I, split=s)), np.invert(I))
        same(ht.bitwise_not(ht.array(I, split=s)), np.invert(I))
    same(ht.invert(ht.array(BOOL1, split=0)), np.invert(BOOL1))
    same(ht.invert(ht.array(np.array([0, 255], dtype=np.uint8))), np.invert(np.array([0, 255], dtype=np.uint8)))
    raises(TypeError, ht.invert, ht.array(A))


def test_left_shift():
    for s in splits(2):
        same(ht.left_shift(ht.array(I, split=s), 1), np.left_shift(I, 1))
        same(ht.array(I, split=s) << 2, I << 2)
    raises(TypeError, ht.left_shift, ht.array(A), 1)


def test_right_shift():
    for s in splits(2):
        same(ht.right_shift(ht.array(I, split=s), 1), np.right_shift(I, 1))
        same(ht.array(I * 8, split=s) >> 2, (I * 8) >> 2)
    raises(TypeError, ht.right_shift, ht.array(A), 1)


def test_neg():
    each_split(A, lambda x, s: close(ht.neg(x), -A))
    each_split(A, lambda x, s: close(-x, -A))
    same(ht.negative(ht.array(I, split=0)), -I)
    raises(TypeError, ht.neg, 1)


def test_pos():
    each_split(A, lambda x, s: close(ht.pos(x), A))
    each_split(A, lambda x, s: close(+x, A))
    raises(TypeError, ht.pos, 1)


def _axes_checks(htfn, npfn, data, dtype_check=None):
    for s in splits(data.ndim):
        x = ht.array(data, split=s)
        for ax in range(data.ndim):
            close(htfn(x, axis=ax), npfn(data, axis=ax), rtol=1e-4)


def test_cumsum():
    d = rng(1).standard_normal((5, 7)).astype(np.float32)
    _axes_checks(ht.cumsum, np.cumsum, d)
    same(ht.cumsum(ht.ones(10, dtype=ht.int32, split=0), 0), np.arange(1, 11))
    out = ht.empty((5, 7), split=0)
    ht.cumsum(ht.array(d, split=0), 0, out=out)
    close(out, np.cumsum(d, 0), rtol=1e-4)
    raises(NotImplementedError, ht.cumsum, ht.ones((2, 2)), axis=None)
    raises(TypeError, ht.cumsum, ht.ones((2, 2)), axis="1")
    raises(ValueError, ht.cumsum, ht.ones((2, 2)), axis=3)


def test_cumprod():
    d = (rng(2).random((4, 6)) + 0.5).astype(np.float64)
    _axes_checks(ht.cumprod, np.cumprod, d)
    same(ht.cumproduct(ht.full((6,), 2, dtype=ht.int64, split=0), 0), 2 ** np.arange(1, 7))
    raises(NotImplementedError, ht.cumprod, ht.ones((2, 2)), axis=None)
    raises(ValueError, ht.cumprod, ht.ones((2, 2)), axis=3)


def test_sum():
    d = rng(3).standard_normal((6, 5, 4)).astype(np.float32)
    for s in splits(3):
        x = ht.array(d, split=s)
        close(ht.sum(x), d.sum(), rtol=1e-4, atol=1e-4)
        for ax in (0, 1, 2, (0, 2), (1, 2)):
            close(ht.sum(x, axis=ax), d.sum(axis=ax), rtol=1e-4, atol=1e-5)
        close(ht.sum(x, axis=1, keepdim=True), d.sum(axis=1, keepdims=True), rtol=1e-4, atol=1e-5)
        close(x.sum(axis=0), d.sum(axis=0), rtol=1e-4, atol=1e-5)
    same(ht.sum(ht.ones(11, dtype=ht.int32, split=0)), 11)
    raises(ValueError, ht.sum, ht.ones((2, 2)), axis=5)
    raises(TypeError, ht.sum, ht.ones((2, 2)), axis="0")


def test_prod():
    d = (rng(4).random((3, 4)) + 0.5)
    for s in splits(2):
        x = ht.array(d, split=s)
        close(ht.prod(x), d.prod(), rtol=1e-10)
        for ax in (0, 1):
            close(ht.prod(x, axis=ax), d.prod(axis=ax), rtol=1e-10)
    same(ht.prod(ht.full((5,), 2, dtype=ht.int64, split=0)), 32)
    raises(ValueError, ht.prod, ht.ones((2, 2)), axis=5)


def test_diff():
    d = rng(5).standard_normal((7, 6))
    for s in splits(2):
        x = ht.array(d, split=s)
        for ax in (0, 1):
            for n in (1, 2, 3):
                close(ht.diff(x, n=n, axis=ax), np.diff(d, n=n, axis=ax), rtol=1e-10, atol=1e-10)
    close(ht.diff(ht.array(d, split=0), n=0), d)
    raises(ValueError, ht.diff, ht.array(d), n=-1)
    raises(TypeError, ht.diff, d)


def test_right_hand_side_operations():
    x = ht.array(A, split=0)
    for op, npop in ((operator.add, np.add), (operator.sub, np.subtract), (operator.mul, np.multiply),
                     (operator.truediv, np.divide), (operator.pow, np.power), (operator.mod, np.mod),
                     (operator.floordiv, np.floor_divide)):
        close(op(3.0, x), npop(np.float32(3.0), A), rtol=1e-5)
        close(op(x, 3.0), npop(A, np.float32(3.0)), rtol=1e-5)
    xi = ht.array(I, split=1)
    for op, npop in ((operator.and_, np.bitwise_and), (operator.or_, np.bitwise_or), (operator.xor, np.bitwise_xor),
                     (operator.lshift, np.left_shift), (operator.rshift, np.right_shift)):
        same(op(3, xi), npop(3, I))
    # torch tensors on the left promote to DNDarrays
    close(torch.tensor(A) + ht.array(A, split=0), A + A)
