"""Parity with ``heat/core/tests/test_dndarray.py``: metadata properties (sizes, bytes, strides,
lshape maps, counts/displs), halos, casts to Python scalars, bitwise operators, balancing,
redistribution to arbitrary target maps, resplit, flatten, fill_diagonal, get/setitem and the
torch proxy, on every split."""
import numpy as np
import torch

import heat_amd as ht

from ._util import close, raises, rng, same, splits


def _world():
    c = ht.MPI_WORLD
    return c, c.size, c.rank


def test_and():
    a = np.array([[1, 2], [3, 4]], dtype=np.int32)
    for s in splits(2):
        same(ht.array(a, split=s) & ht.array(np.array([2, 2], dtype=np.int32)), a & 2)
        same(ht.array(a > 1, split=s) & ht.array(a < 4, split=s), (a > 1) & (a < 4))


def test_or():
    a = np.array([[1, 2], [3, 4]], dtype=np.int32)
    for s in splits(2):
        same(ht.array(a, split=s) | 8, a | 8)


def test_xor():
    a = np.array([[1, 2], [3, 4]], dtype=np.int32)
    for s in splits(2):
        same(ht.array(a, split=s) ^ ht.array(a, split=s), a ^ a)
        same(ht.array(a, split=s) ^ 5, a ^ 5)


def test_invert():
    a = np.array([[1, -2], [3, 0]], dtype=np.int64)
    for s in splits(2):
        same(~ht.array(a, split=s), ~a)
    same(~ht.array(np.array([True, False]), split=0), np.array([False, True]))
    raises(TypeError, lambda: ~ht.array([1.5, 2.0]))


def test_lshift():
    a = np.arange(12, dtype=np.int32).reshape(3, 4)
    for s in splits(2):
        same(ht.array(a, split=s) << 3, a << 3)
        same(ht.array(a, split=s) << ht.array(np.full((4,), 2, dtype=np.int32)), a << 2)
    raises(TypeError, lambda: ht.array([1.0]) << 1)


def test_rshift():
    a = np.arange(12, dtype=np.int32).reshape(3, 4) * 16
    for s in splits(2):
        same(ht.array(a, split=s) >> 3, a >> 3)
    raises(TypeError, lambda: ht.array([1.0]) >> 1)


def test_gethalo():
    comm, p, me = _world()
    data = np.arange(2 * 6 * p).reshape(2, 6 * p)
    x = ht.array(data, split=1)
    x.get_halo(2)
    off, lshape, _ = comm.chunk(x.shape, 1)
    lo, hi = off, off + lshape[1]
    if me > 0:
        assert torch.equal(x.halo_prev.cpu(), torch.tensor(data[:, lo - 2: lo]))
    else:
        assert x.halo_prev is None
    if me < p - 1:
        assert torch.equal(x.halo_next.cpu(), torch.tensor(data[:, hi: hi + 2]))
    else:
        assert x.halo_next is None
    width = lshape[1] + (2 if me > 0 else 0) + (2 if me < p - 1 else 0)
    assert tuple(x.array_with_halos.shape) == (2, width)
    raises(TypeError, x.get_halo, "2")
    raises(ValueError, x.get_halo, -1)
    # split 0, 1-element halo
    y = ht.array(np.arange(4 * p * 3).reshape(4 * p, 3), split=0)
    y.get_halo(1)
    if p > 1 and me == 0:
        assert torch.equal(y.halo_next.cpu(), torch.tensor(np.arange(4 * p * 3).reshape(4 * p, 3)[4:5]))


def test_larray():
    x = ht.arange(10, split=0)
    assert isinstance(x.larray, torch.Tensor)
    x.larray = x.larray * 2
    assert int(ht.sum(x).item()) == 90
    raises(TypeError, setattr, x, "larray", [1, 2, 3])


def test_astype():
    data = np.array([[1.7, -2.2], [3.5, 4.0]], dtype=np.float32)
    for s in splits(2):
        x = ht.array(data, split=s)
        y = x.astype(ht.int32)
        assert y.dtype is ht.int32 and y.larray.dtype == torch.int32
        same(y, data.astype(np.int32))
        z = x.astype(ht.float64, copy=False)
        assert z is x and x.dtype is ht.float64
    b = ht.array([0, 1, 2]).astype(ht.bool)
    same(b, np.array([False, True, True]))


def test_balance_and_lshape_map():
    comm, p, me = _world()
    data = ht.zeros((70, 20), split=0)
    lmap = data.create_lshape_map()
    assert tuple(lmap.shape) == (p, 2)
    assert lmap[:, 0].sum().item() == 70 and torch.all(lmap[:, 1] == 20)
    # unbalance: rank r holds r + 1 rows
    x = ht.array(torch.full((me + 1, 3), float(me)), is_split=0)
    assert x.shape == (p * (p + 1) // 2, 3)
    assert x.is_balanced(force_check=True) == (p <= 2 and p * (p + 1) // 2 % p == 0 and p == 1)
    ref = x.numpy()
    x.balance_()
    assert x.is_balanced(force_check=True)
    same(x, ref)
    y = ht.array(torch.full((2, me + 1), float(me)), is_split=1)
    yb = ht.balance(y, copy=True)
    assert yb.is_balanced()
    same(yb, y.numpy())


def test_bool_cast():
    assert bool(ht.array([1])) is True and bool(ht.array(0.0)) is False
    assert bool(ht.array([[1]], split=0))
    raises(TypeError, bool, ht.array([1, 2]))


def test_complex_cast():
    assert complex(ht.array(2.5)) == 2.5 + 0j
    assert complex(ht.array([[1 + 2j]], split=1)) == 1 + 2j
    raises(TypeError, complex, ht.array([1, 2]))


def test_float_cast():
    assert float(ht.array([2])) == 2.0 and isinstance(float(ht.array([2])), float)
    assert float(ht.array([[3.5]], split=0)) == 3.5
    raises(TypeError, float, ht.array([1, 2], split=0))


def test_int_cast():
    assert int(ht.array([2.9])) == 2
    assert int(ht.array([[7]], split=1)) == 7
    raises(TypeError, int, ht.ones((2, 2)))


def test_counts_displs():
    comm, p, me = _world()
    a = ht.arange(128, split=0).reshape((8, 8, 2))
    counts, displs = a.counts_displs()
    c2, d2, _ = comm.counts_displs_shape(a.gshape, a.split)
    assert tuple(counts) == tuple(c2) and tuple(displs) == tuple(d2)
    b = ht.array(torch.ones(8, 2 * me, 2), is_split=1)
    counts, displs = b.counts_displs()
    assert list(counts) == [2 * r for r in range(p)]
    assert list(displs) == [sum(2 * q for q in range(r)) for r in range(p)]
    raises(ValueError, ht.arange(128).reshape((8, 8, 2)).counts_displs)


def test_flatten():
    d = np.arange(60).reshape(3, 4, 5)
    for s in splits(3):
        f = ht.array(d, split=s).flatten()
        same(f, d.flatten())
        assert f.split == (None if s is None else 0)


def test_fill_diagonal():
    for shape in ((6, 6), (5, 8), (9, 4)):
        for s in splits(2):
            x = ht.zeros(shape, split=s)
            x.fill_diagonal(3)
            ref = np.zeros(shape, dtype=np.float32)
            np.fill_diagonal(ref, 3)
            same(x, ref)


def test_is_balanced():
    comm, p, me = _world()
    assert ht.zeros((10, 3), split=0).is_balanced()
    assert ht.zeros((10, 3)).is_balanced()
    x = ht.array(torch.zeros(me * 2 + 1), is_split=0)
    assert x.is_balanced(force_check=True) == (p == 1)


def test_is_distributed():
    comm, p, me = _world()
    assert not ht.zeros((4, 4)).is_distributed()
    assert ht.zeros((4, 4), split=0).is_distributed() == (p > 1)


def test_item():
    assert ht.zeros((1,)).item() == 0
    assert ht.array([[4]], split=0).item() == 4
    assert isinstance(ht.array(1.5).item(), float)
    raises(ValueError, ht.zeros((2,)).item)


def test_len():
    assert len(ht.zeros((7, 3), split=0)) == 7
    assert len(ht.zeros((7, 3), split=1)) == 7
    raises(TypeError, len, ht.array(3.0))


def test_lloc():
    a = ht.zeros((13, 5), split=0)
    if a.lshape[0] > 7:
        a.lloc[0, 0] = 1
        assert a.larray[0, 0] == 1 and a.lloc[0, 0].dtype == torch.float32
        a.lloc[1:3, 1] = 1
        assert torch.all(a.larray[1:3, 1] == 1)
        a.lloc[3:7:2, 2:5:2] = 1
        assert torch.all(a.larray[3:7:2, 2:5:2] == 1)
    b = ht.zeros((4, 5))
    b.lloc[3:4, 1:5:2] = 2
    assert torch.all(b.larray[3, 1::2] == 2) and b.larray.sum() == 4


def test_lnbytes():
    comm, p, me = _world()
    for dt, es in ((ht.int32, 4), (ht.float64, 8), (ht.int16, 2), (ht.bool, 1)):
        x = ht.zeros((17, 3), dtype=dt, split=0)
        assert x.lnbytes == x.lshape[0] * 3 * es
        assert x.gnbytes == 17 * 3 * es
        assert ht.zeros((17, 3), dtype=dt).lnbytes == 17 * 3 * es


def test_nbytes():
    x = ht.zeros((10, 10), dtype=ht.float32, split=1)
    assert x.nbytes == 400 and x.gnbytes == 400
    assert ht.zeros((3,), dtype=ht.complex64).nbytes == 24


def test_ndim():
    assert ht.zeros((1, 2, 3), split=2).ndim == 3 and ht.array(1).ndim == 0


def test_numpy():
    d = rng(1).standard_normal((11, 4)).astype(np.float32)
    for s in splits(2):
        n = ht.array(d, split=s).numpy()
        assert isinstance(n, np.ndarray) and n.dtype == np.float32
        same(n, d)
    same(np.array(ht.array(d, split=0)), d)


def test_redistribute():
    comm, p, me = _world()
    st = ht.zeros((50,), split=0)
    target = torch.zeros((p, 1), dtype=torch.int64)
    target[p - 1] = 30
    target[0] += 20
    st.redistribute_(target_map=target)
    assert st.lshape == (int(target[me, 0]),)
    same(st, np.zeros(50, dtype=np.float32))
    d = np.arange(50 * 6).reshape(6, 50)
    x = ht.array(d, split=1)
    tgt = torch.tensor([[6, 0]] * p, dtype=torch.int64)
    tgt[0, 1] = 13
    tgt[p - 1, 1] += 50 - 13
    x.redistribute_(lshape_map=x.create_lshape_map(), target_map=tgt)
    assert x.lshape == (6, int(tgt[me, 1]))
    same(x, d)
    raises(TypeError, x.redistribute_, target_map="x")


def test_repr():
    a = ht.array([1, 2, 3, 4])
    assert repr(a) == str(a)
    if a.comm.rank == 0:  # printing gathers to rank 0 only (reference printing.py)
        assert "DNDarray" in repr(a)


def test_resplit():
    comm, p, me = _world()
    data = ht.zeros((p, p), split=None)
    data.resplit_(None)
    assert data.split is None and data.lshape == (p, p)
    d = np.arange(p * 3 * 5).reshape(p * 3, 5)
    for a in splits(2):
        for b in splits(2):
            x = ht.array(d, split=a)
            x.resplit_(b)
            assert x.split == b
            same(x, d)
            y = ht.resplit(ht.array(d, split=a), b)
            same(y, d)
            if b is not None:
                assert y.lshape == comm.chunk(y.shape, b)[1]


def test_rshift_lshift_mixed_dtypes():
    x = ht.array(np.array([8, 16], dtype=np.int64), split=0)
    same(x >> 2, np.array([2, 4]))


def test_setitem_getitem():
    d = np.arange(5 * 6 * 7).reshape(5, 6, 7).astype(np.float32)
    keys = [0, -1, (1, 2), (slice(1, 4), 3), (slice(None), slice(2, 6, 2)), (Ellipsis, 1), (slice(None, None, -1),),
            (np.array([0, 3, 4]),), (slice(None), [5, 1, 2]), (2, slice(None), 6)]
    for s in splits(3):
        x = ht.array(d, split=s)
        for k in keys:
            got = x[k]
            exp = d[k]
            if isinstance(got, ht.DNDarray):
                same(got, exp)
            else:
                assert np.asarray(got) == exp
        same(x[x > 100], d[d > 100])
        y = ht.array(d, split=s)
        e = d.copy()
        y[1:3, :, 2] = -1.0
        e[1:3, :, 2] = -1.0
        y[0] = ht.ones((6, 7))
        e[0] = 1.0
        y[y > 200] = 0
        e[e > 200] = 0
        y[:, [0, 5]] = 9.0
        e[:, [0, 5]] = 9.0
        same(y, e)
    raises(IndexError, lambda: ht.zeros((3, 3), split=0)[5])


def test_size_gnumel():
    x = ht.zeros((10, 11, 12), split=1)
    assert x.size == x.gnumel == 1320
    assert x.lnumel == int(np.prod(x.lshape))
    assert ht.array(3).size == 1


def test_stride_and_strides():
    t = torch.arange(6 * 5 * 4, dtype=torch.int16).reshape(6, 5, 4)
    h = ht.array(t)
    assert h.stride() == t.stride() and h.strides == t.numpy().strides
    tf = torch.arange(6 * 5 * 4, dtype=torch.float64).reshape(6, 5, 4).permute(2, 1, 0)
    hf = ht.array(tf)
    assert hf.stride() == tf.stride() or hf.stride() == tf.contiguous().stride()
    x = ht.zeros((8, 3), dtype=ht.float32, split=0)
    assert x.strides == (12, 4)


def test_tolist():
    d = [[1, 2, 3], [4, 5, 6]]
    for s in splits(2):
        assert ht.array(d, split=s).tolist() == d
    assert ht.array([1.5, 2.5], split=0).tolist() == [1.5, 2.5]


def test_torch_proxy():
    x = ht.array(1)
    px = x.__torch_proxy__()
    assert px.ndim == 0
    y = ht.zeros((10, 3), split=0)
    py = y.__torch_proxy__()
    assert tuple(py.shape) == (10, 3)
    assert py.untyped_storage().nbytes() <= 1
