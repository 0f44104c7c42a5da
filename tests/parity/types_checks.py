"""Parity with ``heat/core/tests/test_types.py``: the type hierarchy (abstract types cannot be
instantiated, concrete types construct DNDarrays), aliases, iscomplex/isreal, canonical_heat_type,
heat_type_of, issubdtype, promotion/result_type tables, can_cast and finfo/iinfo."""
import numpy as np
import torch

import heat_amd as ht

from ._util import raises, same


def _abstract(t):
    assert isinstance(t, type) and issubclass(t, ht.datatype)
    raises(TypeError, t)


def _concrete(t, tt):
    assert isinstance(t, type) and issubclass(t, ht.datatype)
    v = t()
    assert isinstance(v, ht.DNDarray) and v.shape == (1,) and bool((v.larray == 0).all()) and v.larray.dtype == tt
    gt = [[3, 2, 1], [4, 5, 6]]
    v = t(gt)
    assert v.shape == (2, 3) and v.larray.dtype == tt
    assert bool((v.larray.cpu() == torch.tensor(gt, dtype=tt)).all())
    raises(TypeError, t, gt, gt)


def test_generic():
    _abstract(ht.datatype)


def test_bool():
    _concrete(ht.bool, torch.bool)
    _concrete(ht.bool_, torch.bool)


def test_number():
    _abstract(ht.number)


def test_integer():
    _abstract(ht.integer)


def test_signedinteger():
    _abstract(ht.signedinteger)


def test_int8():
    _concrete(ht.int8, torch.int8)
    _concrete(ht.byte, torch.int8)


def test_int16():
    _concrete(ht.int16, torch.int16)
    _concrete(ht.short, torch.int16)


def test_int32():
    _concrete(ht.int32, torch.int32)
    _concrete(ht.int, torch.int32)


def test_int64():
    _concrete(ht.int64, torch.int64)
    _concrete(ht.long, torch.int64)


def test_unsignedinteger():
    _abstract(ht.unsignedinteger)


def test_uint8():
    _concrete(ht.uint8, torch.uint8)
    _concrete(ht.ubyte, torch.uint8)


def test_floating():
    _abstract(ht.floating)


def test_float32():
    _concrete(ht.float32, torch.float32)
    _concrete(ht.float, torch.float32)
    _concrete(ht.float_, torch.float32)


def test_float64():
    _concrete(ht.float64, torch.float64)
    _concrete(ht.double, torch.float64)


def test_flexible():
    _abstract(ht.flexible)


def test_complex64():
    _concrete(ht.complex64, torch.complex64)
    _concrete(ht.cfloat, torch.complex64)
    _concrete(ht.csingle, torch.complex64)
    assert ht.complex64.char() == "c8" and ht.int32.char() == "i4" and ht.float64.char() == "f8"


def test_complex128():
    _concrete(ht.complex128, torch.complex128)
    _concrete(ht.cdouble, torch.complex128)
    assert ht.complex128.char() == "c16"


def _pred(fn, rows):
    for data, expect, split in rows:
        r = fn(ht.array(data, split=split) if not isinstance(data, ht.DNDarray) else data)
        assert r.dtype == ht.bool and r.shape == np.shape(expect)
        same(r, expect)


def test_iscomplex():
    _pred(ht.iscomplex, [([1, 1.2, 1 + 1j, 1 + 0j], [False, False, True, False], None),
                         ([1, 1.2, True], [False, False, False], 0),
                         (ht.ones((6, 6), dtype=ht.bool, split=0), np.zeros((6, 6), bool), 0),
                         # a complex fill value makes the array complex whatever dtype says (reference)
                         (ht.full((5, 5), 1 + 1j, dtype=ht.int, split=1), np.ones((5, 5), bool), 1)])


def test_isreal():
    _pred(ht.isreal, [([1, 1.2, 1 + 1j, 1 + 0j], [True, True, False, True], None),
                      ([1, 1.2, True], [True, True, True], 0),
                      (ht.ones((6, 6), dtype=ht.bool, split=0), np.ones((6, 6), bool), 0),
                      (ht.full((5, 5), 1 + 1j, dtype=ht.int, split=1), np.zeros((5, 5), bool), 1)])


def test_can_cast():
    assert ht.can_cast(ht.int8, ht.int16) and ht.can_cast(ht.int32, ht.float64)
    assert not ht.can_cast(ht.float64, ht.int32) and ht.can_cast(ht.float64, ht.int32, casting="unsafe")
    assert ht.can_cast(ht.int64, ht.int8, casting="same_kind") and not ht.can_cast(ht.float32, ht.int8, casting="same_kind")
    assert ht.can_cast(ht.float64, ht.float32, casting="same_kind")
    assert not ht.can_cast(ht.float64, ht.float32, casting="safe")
    assert ht.can_cast(ht.int32, ht.int32, casting="no") and not ht.can_cast(ht.int32, ht.int64, casting="no")
    assert ht.can_cast(1, ht.int8) and ht.can_cast(ht.zeros(3, dtype=ht.int8), ht.int16)
    raises(TypeError, ht.can_cast, ht.int32, ht.int32, casting=1)
    raises(ValueError, ht.can_cast, ht.int32, ht.int32, casting="hello")
    raises(TypeError, ht.can_cast, {}, ht.int32)


def test_canonical_heat_type():
    c = ht.core.types.canonical_heat_type
    assert c(ht.float32) == ht.float32 and c("?") == ht.bool and c(int) == ht.int32
    assert c("u1") == ht.uint8 and c(np.int8) == ht.int8 and c(torch.short) == ht.int16
    assert c(torch.cfloat) == ht.complex64
    for bad in ({}, object, 1, "i7"):
        raises(TypeError, c, bad)


def test_heat_type_of():
    f = ht.core.types.heat_type_of
    assert f(ht.zeros((1,), dtype=ht.bool)) == ht.bool
    assert f(np.ones((3,), dtype=np.int32)) == ht.int32
    assert f(2.0) == ht.float32
    assert f([3, "hello world"]) == ht.int32
    assert f(torch.full((2,), 1 + 1j, dtype=torch.complex128)) == ht.complex128
    raises(TypeError, f, {})
    raises(TypeError, f, object)


def test_issubdtype():
    for t in (ht.bool, ht.bool_, ht.number, ht.integer, ht.signedinteger, ht.unsignedinteger, ht.floating,
              ht.flexible):
        assert ht.issubdtype(t, ht.datatype)
    for a, b in ((ht.integer, ht.number), (ht.floating, ht.number), (ht.signedinteger, ht.integer),
                 (ht.unsignedinteger, ht.integer), (ht.int8, ht.signedinteger), (ht.int16, ht.signedinteger),
                 (ht.int32, ht.signedinteger), (ht.int64, ht.signedinteger), (ht.uint8, ht.unsignedinteger),
                 (ht.float32, ht.floating), (ht.float64, ht.floating), (ht.byte, ht.int8), (ht.short, ht.int16),
                 (ht.int, ht.int32), (ht.long, ht.int64), (ht.uint8, ht.ubyte), (ht.float32, ht.float),
                 (ht.float32, ht.float_), (ht.float64, ht.double), ("B", ht.uint8), (ht.float64, "f8")):
        assert ht.issubdtype(a, b), (a, b)
    assert not ht.issubdtype(ht.float32, ht.integer) and not ht.issubdtype(ht.int8, ht.floating)
    raises(TypeError, ht.issubdtype, ht.bool, True)
    raises(TypeError, ht.issubdtype, 4.2, "f")
    raises(TypeError, ht.issubdtype, {}, ht.int)


def test_type_promotions():
    assert ht.promote_types(ht.uint8, ht.uint8) == ht.uint8
    assert ht.promote_types(ht.int8, ht.uint8) == ht.int16
    assert ht.promote_types(ht.int32, ht.float32) == ht.float32
    assert ht.promote_types("f4", ht.float) == ht.float32
    assert ht.promote_types(ht.bool_, "?") == ht.bool
    assert ht.promote_types(ht.float32, ht.complex64) == ht.complex64
    # symmetric on every pair
    ts = [ht.bool, ht.uint8, ht.int8, ht.int16, ht.int32, ht.int64, ht.float32, ht.float64, ht.complex64, ht.complex128]
    for a in ts:
        for b in ts:
            assert ht.promote_types(a, b) == ht.promote_types(b, a)
    raises(TypeError, ht.promote_types, 1, "?")
    raises(TypeError, ht.promote_types, ht.float32, "hello world")


def test_result_type():
    assert ht.result_type(1) == ht.int32
    assert ht.result_type(1, 1.0) == ht.float32
    assert ht.result_type(1.0, True, 1 + 1j) == ht.complex64
    assert ht.result_type(ht.array(1, dtype=ht.int32), 1) == ht.int32
    assert ht.result_type(1.0, ht.array(1, dtype=ht.int32)) == ht.float32
    assert ht.result_type(ht.uint8, ht.int8) == ht.int16
    assert ht.result_type("b", "f4") == ht.float32
    assert ht.result_type(ht.array([1], dtype=ht.float64), "f4") == ht.float64
    assert ht.result_type(ht.array([1, 2, 3, 4], dtype=ht.float64, split=0), 1, ht.bool, "u", torch.uint8,
                          np.complex128, ht.array(1, dtype=ht.int64)) == ht.complex128
    assert ht.result_type(np.array([1, 2, 3]), np.dtype("int32"), torch.tensor([1, 2, 3])) == ht.int64


def test_finfo():
    i = ht.finfo(ht.float32)
    assert i.bits == 32 and i.max == (2 - 2 ** -23) * 2 ** 127 and i.min == -i.max and i.eps == 2 ** -23
    i = ht.finfo(ht.float64)
    assert i.bits == 64 and i.eps == 2 ** -52
    raises(TypeError, ht.finfo, 1)
    raises(TypeError, ht.finfo, ht.int32)
    raises(TypeError, ht.finfo, "float16")


def test_iinfo():
    i = ht.iinfo(ht.int32)
    assert i.bits == 32 and i.max == 2147483647 and i.min == -2147483648
    assert ht.iinfo(ht.uint8).max == 255 and ht.iinfo(ht.int64).bits == 64
    raises(TypeError, ht.iinfo, 1.0)
    raises(TypeError, ht.iinfo, ht.float64)
    raises(TypeError, ht.iinfo, "int16")
