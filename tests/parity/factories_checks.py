"""Parity with ``heat/core/tests/test_factories.py``: every factory's shape/lshape/split/dtype,
values against NumPy, ``is_split`` assembly (uneven blocks, ndmin), copy semantics, the
``*_like`` variants, meshgrid splits and all the TypeErrors/ValueErrors."""
import numpy as np
import torch

import heat_amd as ht

from ._util import close, raises, same, splits


def _chunk_ok(a):
    if a.split is None:
        assert a.lshape == a.gshape
    else:
        for i, (g, l) in enumerate(zip(a.gshape, a.lshape)):
            assert (l <= g) if i == a.split else (l == g)


def test_arange():
    cases = [((10,), {}, np.arange(10), ht.int32), ((0, 10), {}, np.arange(0, 10), ht.int32),
             ((0, 10, 2), {}, np.arange(0, 10, 2), ht.int32), ((0, 10, 2.0), {}, np.arange(0, 10, 2.0), ht.float32),
             ((0, 10, 2.0), {"dtype": torch.int16}, np.arange(0, 10, 2), ht.int16),
             ((0, 10, 2), {"dtype": torch.float64}, np.arange(0, 10, 2.0), ht.float64),
             ((-5, 3, 0.7), {}, np.arange(-5, 3, 0.7), ht.float32), ((10, 0, -3), {}, np.arange(10, 0, -3), ht.int32)]
    for args, kw, expected, dt in cases:
        for s in (None, 0):
            a = ht.arange(*args, split=s, **kw)
            assert a.dtype == dt and a.split == s and a.shape == expected.shape, (args, a.dtype, a.shape)
            _chunk_ok(a)
            close(a, expected, rtol=1e-6)
    assert int(ht.arange(0, 10, 2).sum().item()) == 20
    raises(ValueError, ht.arange, -5, 3, split=1)
    raises(TypeError, ht.arange)
    raises(TypeError, ht.arange, 1, 2, 3, 4)


def test_array():
    a = ht.array([[1, 2, 3], [4, 5, 6]])
    assert a.dtype == ht.int64 and a.lshape == (2, 3) and a.split is None
    b = ht.array(((0, 0), (1, 1)), dtype=ht.int8)
    assert b.dtype == ht.int8 and b.larray.dtype == torch.int8
    t = torch.tensor([6, 5, 4, 3, 2, 1])
    c = ht.array(t, copy=False)
    assert c.dtype == ht.int64 and c.larray is t
    c2 = ht.array(t)
    assert c2.larray is not t and c2.larray.data_ptr() != t.data_ptr()
    d = ht.array([4.0, 5.0, 6.0], ndmin=3)
    assert d.dtype == ht.float32 and d.gshape == (3, 1, 1)
    d = ht.array([4.0, 5.0, 6.0], ndmin=-3)
    assert d.gshape == (1, 1, 3)
    t2 = ht.array([[1.0, 2.0, 3.0]] * 3, split=0)
    assert t2.dtype == ht.float32 and t2.gshape == (3, 3) and t2.split == 0
    _chunk_ok(t2)
    assert (t2.larray.cpu() == torch.tensor([1.0, 2.0, 3.0])).all()
    x = np.arange(60.0).reshape(3, 4, 5)
    for s in splits(3):
        h = ht.array(x, split=s)
        _chunk_ok(h)
        same(h, x)
    # is_split: uneven per-rank blocks, ndmin padding, global shape from all ranks
    rank, size = ht.MPI_WORLD.rank, ht.MPI_WORLD.size
    data = [[4.0, 5.0, 6.0], [1.0, 2.0, 3.0], [0.0, 0.0, 0.0]] if rank == 0 else [[4.0, 5.0, 6.0], [1.0, 2.0, 3.0]]
    e = ht.array(data, ndmin=3, is_split=0)
    assert e.dtype == ht.float32 and e.split == 0
    assert e.lshape == ((3, 3, 1) if rank == 0 else (2, 3, 1))
    assert e.gshape == (3 + 2 * (size - 1), 3, 1)
    data = [[4.0, 5.0, 6.0], [1.0, 2.0, 3.0]]
    e = ht.array(data, ndmin=-3, is_split=1)
    assert e.gshape == (1, 2 * size, 3) and e.lshape == (1, 2, 3) and e.split == 1
    blk = np.full((rank + 1, 2), rank, dtype=np.float64)
    f = ht.array(blk, is_split=0)
    expect = np.concatenate([np.full((r + 1, 2), r, dtype=np.float64) for r in range(size)])
    same(f, expect)
    if size > 1:
        bad = [4.0, 5.0, 6.0] if rank == 0 else [[4.0, 5.0, 6.0], [1.0, 2.0, 3.0]]
        raises(ValueError, ht.array, bad, is_split=0)
        bad = [[4.0, 5.0, 6.0], [1.0, 2.0, 3.0], [0.0, 0.0, 0.0]] if rank == 0 else [[4.0, 5.0, 6.0], [1.0, 2.0, 3.0]]
        raises(ValueError, ht.array, bad, is_split=1)
    raises(ValueError, ht.array, [[1.0, 2.0, 3.0], [1.0, 2.0, 3.0]], split=0, is_split=0)
    raises(TypeError, ht.array, map)
    raises(TypeError, ht.array, "abc")
    raises(TypeError, ht.array, (4,), dtype="a")
    raises(TypeError, ht.array, (4,), ndmin=3.0)
    raises(TypeError, ht.array, (4,), split="a")
    raises(ValueError, ht.array, (4,), split=3)
    raises(TypeError, ht.array, (4,), comm={})


def test_asarray():
    arr = ht.array([1, 2])
    assert ht.asarray(arr) is arr
    arr = ht.array([1, 2, 3, 4, 5, 6], split=0)
    lst = arr.tolist(keepsplit=True)
    asarr = ht.asarray(lst, is_split=0)
    assert asarr.shape == arr.shape and asarr.split == 0 and ht.equal(asarr, arr)
    n = np.array([1, 2, 3, 4])
    asarr = ht.asarray(n)
    same(asarr, n)
    asarr[0] = 0
    if asarr.device == ht.cpu:
        assert n[0] == 0  # shares memory with the NumPy array on the host
    t = torch.tensor([1, 2, 3, 4])
    asarr = ht.asarray(t)
    assert torch.equal(asarr.larray, t)
    asarr[0] = 0
    assert t[0].item() == 0


def _basic_factory(fn, value, **kw):
    a = fn(3, **kw)
    assert a.shape == (3,) and a.lshape == (3,) and a.split is None and a.dtype == ht.float32
    a = fn(5, dtype=ht.bool, **kw)
    assert a.dtype == ht.bool
    a = fn((2, 3), dtype=ht.int32, **kw)
    assert a.shape == (2, 3) and a.dtype == ht.int32
    for s in splits(2):
        a = fn((6, 4), dtype=ht.int32, split=s, **kw)
        assert a.shape == (6, 4) and a.split == s and a.dtype == ht.int32
        _chunk_ok(a)
        if value is not None:
            same(a, np.full((6, 4), value, dtype=np.int32))
    a = fn((7, 3, 2), split=-1, **kw)
    assert a.split == 2
    raises(TypeError, fn, "(2, 3,)", dtype=ht.float64, **kw)
    raises(ValueError, fn, (-1, 3), dtype=ht.float64, **kw)
    raises(TypeError, fn, (2, 3), dtype=ht.float64, split="axis", **kw)


def test_empty():
    _basic_factory(ht.empty, None)


def test_zeros():
    _basic_factory(ht.zeros, 0)


def test_ones():
    _basic_factory(ht.ones, 1)


def test_full():
    _basic_factory(lambda shape, **kw: ht.full(shape, 4, **kw), 4)
    a = ht.full((2, 3), 7.5, dtype=ht.float64, split=0)
    same(a, np.full((2, 3), 7.5))


def _like(fn, value, **kw):
    for s in splits(2):
        base = ht.zeros((5, 4), dtype=ht.int32, split=s)
        a = fn(base, **kw)
        assert a.shape == (5, 4) and a.split == s and a.dtype == ht.int32
        _chunk_ok(a)
        if value is not None:
            same(a, np.full((5, 4), value, dtype=np.int32))
        a = fn(base, dtype=ht.float64, **kw)
        assert a.dtype == ht.float64
        # split=None inherits the prototype's split (reference factories.py __factory_like)
        a = fn(base, split=None, **kw)
        assert a.split == s
        a = fn(base, split=1, **kw)
        assert a.split == 1
    a = fn([[1, 2], [3, 4]], **kw)
    assert a.shape == (2, 2)
    base = ht.ones((2, 2))
    raises(TypeError, fn, base, dtype="abc", **kw)
    raises(TypeError, fn, base, split="axis", **kw)


def test_empty_like():
    _like(ht.empty_like, None)


def test_zeros_like():
    _like(ht.zeros_like, 0)


def test_ones_like():
    _like(ht.ones_like, 1)


def test_full_like():
    _like(lambda a, dtype=ht.int32, **kw: ht.full_like(a, 4, dtype=dtype, **kw), 4)
    # full_like's default dtype is float32 whatever the prototype, like the reference
    assert ht.full_like(ht.zeros((2, 2), dtype=ht.int64), 3).dtype == ht.float32


def test_eye():
    for shape in (3, (3,), (4, 6), (6, 4), (5, 5)):
        n = (shape, shape) if isinstance(shape, int) else (tuple(shape) if len(shape) > 1 else (shape[0], shape[0]))
        for s in splits(2):
            for dt in (ht.float32, ht.int32, ht.bool):
                e = ht.eye(shape, dtype=dt, split=s)
                assert e.gshape == n and e.split == s and e.dtype == dt
                _chunk_ok(e)
                same(e, np.eye(*n, dtype=dt.char() if hasattr(dt, "char") else None).astype(
                    {ht.float32: np.float32, ht.int32: np.int32, ht.bool: bool}[dt]))
    raises(TypeError, ht.eye, "3")
    raises(ValueError, ht.eye, (-1, 3))


def _spaced(fn, npfn):
    for s in (None, 0):
        a = fn(-3, 5, num=7, split=s)
        assert a.shape == (7,) and a.split == s and a.dtype == ht.float32
        _chunk_ok(a)
        close(a, npfn(-3, 5, num=7), rtol=1e-5)
        a = fn(-3, 5, num=9, endpoint=False, split=s, dtype=ht.float64)
        assert a.dtype == ht.float64
        close(a, npfn(-3, 5, num=9, endpoint=False), rtol=1e-12)
    raises(ValueError, fn, -5, 3, split=1)
    raises(ValueError, fn, -5, 3, num=-1)
    raises(ValueError, fn, -5, 3, num=0)


def test_linspace():
    _spaced(ht.linspace, np.linspace)
    r, step = ht.linspace(-5, 3, num=9, retstep=True)
    assert step == 1.0
    same(r, np.linspace(-5, 3, 9).astype(np.float32))


def test_logspace():
    _spaced(ht.logspace, np.logspace)
    close(ht.logspace(0, 3, num=4, base=2.0), np.logspace(0, 3, num=4, base=2.0))


def test_meshgrid():
    xx, = ht.meshgrid(ht.arange(4))
    same(xx, np.arange(4))
    x, y = ht.arange(4), ht.arange(3)
    xx, yy = ht.meshgrid(x, y)
    nx, ny = np.meshgrid(np.arange(4), np.arange(3))
    assert xx.dtype == x.dtype and yy.dtype == y.dtype
    same(xx, nx)
    same(yy, ny)
    x, y = ht.linspace(0, 4, 3), ht.linspace(0, 4, 5)
    xx, yy = ht.meshgrid(x, y, indexing="ij")
    nx, ny = np.meshgrid(x.numpy(), y.numpy(), indexing="ij")
    same(xx, nx)
    same(yy, ny)
    z = ht.linspace(0, 1, 3, split=0)
    for order in ((0, 1, 2), (1, 0, 2), (1, 2, 0)):
        arrs = [[z, x, y][i] for i in order]
        for ind in ("xy", "ij"):
            res = ht.meshgrid(*arrs, indexing=ind)
            npres = np.meshgrid(*[a.numpy() for a in arrs], indexing=ind)
            splits_seen = {r.split for r in res}
            assert len(splits_seen) == 1 and None not in splits_seen or z.comm.size == 1
            for r, e in zip(res, npres):
                same(r, e)
    raises(ValueError, ht.meshgrid, ht.array(1), indexing="abc")
    raises(ValueError, ht.meshgrid, ht.array([0, 1], split=0), ht.array([1, 2], split=0))
