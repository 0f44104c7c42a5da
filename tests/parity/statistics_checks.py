"""Parity with ``heat/core/tests/test_statistics.py``: every statistic against NumPy/SciPy on
every split, output splits and dtypes, empty local blocks, ``out=`` buffers and error cases."""
import os
from itertools import combinations

import numpy as np
import torch
from scipy import stats as ss

import heat_amd as ht

from ._util import close, raises, rng, same, splits

IRIS = "/root/reference/heat/datasets/iris.csv"


def _iris(split):
    """The reference's iris fixture (a plain CSV) when it is present, else None."""
    if not os.path.exists(IRIS):
        return None
    return ht.load(IRIS, sep=";", split=split)


def _split_after(split, ax):
    if split is None or ax == split:
        return None
    return split if ax > split else split - 1


def _argext_common(fn, npfn, torchfn, tri):
    data = ht.array(rng(1).standard_normal((3, 4, 5)).astype(np.float32))
    r = fn(data, axis=0)
    assert r.dtype == ht.int64 and r.larray.dtype == torch.int64
    assert r.shape == (4, 5) and r.lshape == (4, 5) and r.split is None
    assert torch.equal(r.larray, torchfn(data.larray, 0))
    r = fn(data, axis=-1, keepdim=True)
    assert r.shape == (3, 4, 1) and r.split is None
    assert torch.equal(r.larray, torchfn(data.larray, -1, keepdim=True))
    r = fn(data)
    assert r.shape == (1,) or r.shape == (), r.shape
    assert int(r.item()) == int(npfn(data.numpy()))

    v = ht.arange(-10, 10, split=0)
    r = fn(v)
    assert r.split is None and int(r.item()) == int(npfn(np.arange(-10, 10)))

    # is_split: every rank contributes a 4x5 block
    loc = torch.as_tensor(rng(2 + v.comm.rank).standard_normal((4, 5)).astype(np.float32))
    d = ht.array(loc, is_split=0)
    r = fn(d, axis=1)
    assert r.shape == (v.comm.size * 4,) and r.lshape == (4,) and r.split == 0
    assert torch.equal(r.larray, torchfn(loc, 1))

    size = v.comm.size * 2
    d = tri(ht.ones((size, size), split=0))
    expect = npfn(d.numpy(), axis=0)
    r = fn(d, axis=0)
    assert r.shape == (size,) and r.split is None
    same(r, expect)
    out = ht.empty((size,), dtype=ht.int64)
    res = fn(d, axis=0, out=out)
    assert out.dtype == ht.int64 and out.shape == (size,) and out.split is None
    same(out, expect)

    raises(TypeError, fn, d, axis=(0, 1))
    raises(TypeError, fn, d, axis=1.1)
    raises(TypeError, fn, d, axis="y")
    raises(ValueError, fn, d, axis=-4)
    del res


def test_argmax():
    _argext_common(ht.argmax, np.argmax, torch.argmax, lambda a: ht.tril(a, k=-1))
    size = ht.MPI_WORLD.size * 2
    d = ht.tril(ht.ones((size, size), split=0), k=-1)
    raises(TypeError, ht.argmax, d, axis=0, out=ht.empty((size,), dtype=ht.float32))
    # every split, empty blocks included
    x = rng(3).standard_normal((3, 11, 2)).astype(np.float32)
    for s in splits(3):
        for ax in (None, 0, 1, 2):
            same(ht.argmax(ht.array(x, split=s), axis=ax), np.argmax(x, axis=ax).reshape(-1) if ax is None
                 else np.argmax(x, axis=ax))


def test_argmin():
    _argext_common(ht.argmin, np.argmin, torch.argmin, lambda a: ht.triu(a, k=1))
    x = rng(4).standard_normal((3, 11, 2)).astype(np.float32)
    for s in splits(3):
        for ax in (None, 0, 1, 2):
            same(ht.argmin(ht.array(x, split=s), axis=ax), np.argmin(x, axis=ax).reshape(-1) if ax is None
                 else np.argmin(x, axis=ax))


def test_average():
    data = [[1, 2, 3], [4, 5, 6], [7, 8, 9], [10, 11, 12]]
    comp = np.asarray(data, dtype=np.float64)
    for s in splits(2):
        a = ht.array(data, dtype=float, split=s)
        avg = ht.average(a)
        assert avg.shape == () and avg.split is None and avg.dtype == ht.float32
        close(avg, np.average(comp))
        for ax in (0, 1):
            r = ht.average(a, axis=ax)
            assert r.dtype == ht.float32 and r.split == _split_after(s, ax)
            close(r, np.average(comp, axis=ax))

    size = ht.MPI_WORLD.size
    vol = rng(5).standard_normal((3, 3 * size, 3))
    w = rng(6).standard_normal(3 * size)
    for s in splits(3):
        hv = ht.array(vol, split=s)
        for ws in (None, 0):
            r = ht.average(hv, weights=ht.array(w, split=ws), axis=1)
            assert r.shape == (3, 3) and r.dtype == ht.float64 and r.split == _split_after(s, 1)
            close(r, np.average(vol, weights=w, axis=1), rtol=1e-9, atol=1e-9)
        avg, cw = ht.average(hv, weights=ht.array(w), axis=1, returned=True)
        assert isinstance(cw, ht.DNDarray) and cw.gshape == avg.gshape and cw.split == avg.split
        close(cw, np.broadcast_to(w.sum(), (3, 3)), rtol=1e-9, atol=1e-9)
    # full-shape weights with the data's split
    w3 = rng(7).standard_normal(vol.shape)
    for s in splits(3):
        r = ht.average(ht.array(vol, split=s), weights=ht.array(w3, split=s), axis=1)
        close(r, np.average(vol, weights=w3, axis=1), rtol=1e-8, atol=1e-8)
    # tuple axis keeps the remaining split
    rv = ht.array(rng(8).standard_normal((3, 3, 3)).astype(np.float32), split=0)
    r = ht.average(rv, axis=(1, 2))
    assert r.shape == (3,) and r.split == 0 and r.lshape[0] == rv.lshape[0] and r.dtype == ht.float32

    r5 = ht.array(rng(9).standard_normal((size, 2, 3, 4, 5)).astype(np.float32), split=0)
    rw = ht.array(rng(10).standard_normal(size).astype(np.float32), split=0)
    a5 = r5.average(weights=rw, axis=0)
    assert a5.gshape == (2, 3, 4, 5) and a5.split is None and a5.dtype == ht.float32
    close(a5, np.average(r5.numpy(), weights=rw.numpy(), axis=0), rtol=1e-4, atol=1e-4)

    raises(TypeError, ht.average, comp)
    raises(TypeError, ht.average, r5, weights=rw.numpy(), axis=0)
    raises(TypeError, ht.average, r5, weights=rw, axis=None)
    raises(NotImplementedError, ht.average, r5, weights=rw, axis=(1, 2))
    raises(TypeError, ht.average, r5, weights=ht.ones((size, 2)), axis=0)
    raises(ValueError, ht.average, r5, weights=ht.ones(size + 1), axis=0)
    raises(ZeroDivisionError, ht.average, r5, weights=ht.zeros(size, split=0), axis=0)
    raises(NotImplementedError, ht.average, r5, weights=ht.ones(r5.gshape, split=-1), axis=0)
    a = ht.array(data, dtype=float)
    raises(TypeError, a.average, axis=1.1)
    raises(TypeError, a.average, axis="y")
    raises(ValueError, ht.average, a, axis=-4)


def test_bincount():
    r = ht.bincount(ht.array([], dtype=ht.int))
    assert r.size == 0 and r.dtype == ht.int64
    for s in (None, 0):
        a = ht.arange(5, split=s)
        r = ht.bincount(a)
        assert r.dtype == ht.int64 and ht.equal(r, ht.ones((5,), dtype=ht.int64))
        r = ht.bincount(a, weights=ht.arange(5, split=s))
        assert r.dtype == ht.float64 and ht.equal(r, ht.arange(5, dtype=ht.float64))
        r = ht.bincount(a, minlength=8)
        same(r, np.array([1, 1, 1, 1, 1, 0, 0, 0]))
    x = rng(11).integers(0, 9, 37)
    w = rng(12).standard_normal(37)
    for s in (None, 0):
        same(ht.bincount(ht.array(x, split=s)), np.bincount(x))
        close(ht.bincount(ht.array(x, split=s), weights=ht.array(w, split=s)), np.bincount(x, weights=w))
    raises(ValueError, ht.bincount, ht.array([0, 1, 2, 3], split=0), weights=ht.array([1, 2, 3, 4]))


def test_cov():
    x = ht.array([[0, 2], [1, 1], [2, 0]], dtype=ht.float, split=1).T
    same(ht.cov(x), np.array([[1.0, -1.0], [-1.0, 1.0]], dtype=np.float32))
    data = rng(13).standard_normal((150, 4)) * np.array([0.8, 0.4, 1.7, 0.7]) + np.array([5.8, 3.0, 3.7, 1.2])
    iris = _iris(None)
    if iris is not None:
        data = iris.numpy().astype(np.float64)
    for s in (None, 0, 1):
        hd = ht.array(data.astype(np.float32), split=s)
        close(ht.cov(hd[:, 0], hd[:, 1:3], rowvar=False), np.cov(data[:, 0], data[:, 1:3], rowvar=False), atol=1e-4)
        close(ht.cov(hd, rowvar=False), np.cov(data, rowvar=False), atol=1e-4)
        close(ht.cov(hd, rowvar=False, ddof=1), np.cov(data, rowvar=False, ddof=1), atol=1e-4)
        close(ht.cov(hd, rowvar=False, bias=True), np.cov(data, rowvar=False, bias=True), atol=1e-4)
    small = data[:12]
    for s in (None, 0):
        hs = ht.array(small.astype(np.float32), split=s)
        close(ht.cov(hs, hs, rowvar=True), np.cov(small, small, rowvar=True), atol=1e-4)
    hd = ht.array(data.astype(np.float32), split=0)
    raises(TypeError, ht.cov, data)
    raises(TypeError, ht.cov, hd, data)
    raises(TypeError, ht.cov, hd, ddof="str")
    raises(ValueError, ht.cov, ht.zeros((1, 2, 3)))
    raises(ValueError, ht.cov, hd, ht.zeros((1, 2, 3)))
    raises(ValueError, ht.cov, hd, ddof=10000)


def test_histc():
    c = torch.arange(4, dtype=torch.float64)
    r = ht.histc(ht.array(c), 7)
    assert r.shape == (7,) and r.dtype == ht.float64
    assert torch.equal(r.larray.cpu(), torch.histc(c, 7))
    c = torch.as_tensor(rng(14).random((10, 10, 10)).astype(np.float32))
    comp = torch.histc(c)
    for s in splits(3):
        r = ht.histc(ht.array(c, split=s))
        assert r.shape == (100,) and r.dtype == ht.float32 and r.split is None
        assert torch.equal(r.larray.cpu(), comp), s
    c = torch.as_tensor(rng(15).integers(0, 10, 8).astype(np.float32))
    comp = torch.histc(c, bins=20, min=0, max=20)
    for s in (None, 0):
        out = ht.empty(20, dtype=ht.float32)
        ht.histc(ht.array(c, split=s), bins=20, min=0, max=20, out=out)
        assert out.shape == (20,) and torch.equal(out.larray.cpu(), comp)
    a = ht.arange(10, dtype=ht.float)
    assert ht.equal(ht.histogram(a), ht.histc(a, 10))
    raises(NotImplementedError, ht.histogram, a, "str")
    raises(NotImplementedError, ht.histogram, a, [1, 2, 3])
    raises(NotImplementedError, ht.histogram, a, weights=[1, 2, 3])
    raises(NotImplementedError, ht.histogram, a, normed=True)
    raises(NotImplementedError, ht.histogram, a, density=True)


def _moment_check(fn, ssfn, unbiased_kw):
    x = ht.zeros((2, 3, 4))
    raises(ValueError, fn, x, axis=10)
    raises(TypeError, fn, x, axis="01")
    d1 = rng(16).random(50).astype(np.float32)
    for s in (None, 0):
        assert abs(float(fn(ht.array(d1, split=s))) - ssfn(d1.astype(np.float64), bias=False)) < 1e-4
    d2 = rng(17).random((50, 30))
    for dt in (np.float32, np.float64):
        for s in splits(2):
            h = ht.array(d2.astype(dt), split=s)
            assert abs(float(fn(h)) - ssfn(d2, axis=None, bias=False)) < 1e-4
            for ax in range(2):
                r = fn(h, axis=ax, unbiased=False)
                close(r, ssfn(d2, axis=ax, bias=True), atol=1e-4, rtol=1e-4)
                assert r.split == _split_after(s, ax)
                assert r.dtype == (ht.float64 if dt == np.float64 else ht.float32)
                close(fn(h, axis=ax), ssfn(d2, axis=ax, bias=False), atol=1e-4, rtol=1e-4)
    d3 = rng(18).random((11, 7, 6)).astype(np.float32)
    for s in splits(3):
        h = ht.array(d3, split=s)
        for ax in range(3):
            r = fn(h, axis=ax)
            close(r, ssfn(d3.astype(np.float64), axis=ax, bias=False), atol=1e-4, rtol=1e-4)
            assert r.split == _split_after(s, ax)


def test_kurtosis():
    _moment_check(ht.kurtosis, ss.kurtosis, "unbiased")
    raises(TypeError, ht.kurtosis, ht.zeros((2, 3, 4)), axis=(0, "10"))
    d = rng(19).random((40, 5))
    for s in splits(2):
        close(ht.kurtosis(ht.array(d, split=s), axis=0, Fischer=False),
              ss.kurtosis(d, axis=0, bias=False, fisher=False), atol=1e-8, rtol=1e-8)


def test_skew():
    _moment_check(ht.skew, ss.skew, "unbiased")
    raises(TypeError, ht.zeros((2, 3, 4)).skew, axis=[1, 0])
    assert float(ht.arange(1, 5).skew()) == 0.0


def _ext_common(fn, tfn, npfn, empty_expect):
    data = [[1, 2, 3], [4, 5, 6], [7, 8, 9], [10, 11, 12]]
    comp = torch.tensor(data)
    a = ht.array(data)
    r = fn(a)
    assert r.split is None and r.dtype == ht.int64 and int(r.item()) == int(tfn(comp))
    for dt, tt in ((ht.int8, torch.int8), (ht.int16, torch.int16), (ht.int64, torch.int64)):
        a = ht.array(data, dtype=dt)
        r = fn(a, axis=0)
        assert r.shape == (3,) and r.split is None and r.dtype == dt and r.larray.dtype == tt
        assert torch.equal(r.larray.cpu().long(), tfn(comp, dim=0)[0])
        r = fn(a, axis=1, keepdim=True)
        assert r.shape == (4, 1) and torch.equal(r.larray.cpu().long(), tfn(comp, dim=1, keepdim=True)[0])
    size = ht.MPI_WORLD.size
    v = rng(20).standard_normal((3, 3 * size, 3)).astype(np.float32)
    r = fn(ht.array(v, split=1), axis=1)
    assert r.shape == (3, 3) and r.lshape == (3, 3) and r.split is None and r.dtype == ht.float32
    same(r, npfn(v, axis=1))
    v = rng(21).standard_normal((3 * size, 3, 3)).astype(np.float32)
    h = ht.array(v, split=0)
    r, r2 = fn(h, axis=(1, 2)), fn(h, axis=(2, 1))
    assert r.shape == (3 * size,) and r.split == 0 and (r == r2).all()
    same(r, npfn(v, axis=(1, 2)))
    v5 = rng(22).standard_normal((size, 2, 3, 4, 5)).astype(np.float32)
    r = fn(ht.array(v5, split=0), axis=1)
    assert r.shape == (size, 3, 4, 5) and r.split == 0
    same(r, npfn(v5, axis=1))
    if size > 1:
        r = fn(ht.arange(size - 1, split=0))
        assert int(r.item()) == empty_expect(size)
    # every split and axis with empty blocks
    x = rng(23).standard_normal((2, 3, 9)).astype(np.float32)
    for s in splits(3):
        for ax in (None, 0, 1, 2, (0, 2)):
            # a full reduction has shape (1,) like the reference (_operations.py:416-417)
            same(fn(ht.array(x, split=s), axis=ax), npfn(x, axis=ax).reshape((1,) if ax is None else npfn(x, axis=ax).shape))
    a = ht.array(data)
    raises(TypeError, fn, a, axis=1.1)
    raises(TypeError, fn, a, axis="y")
    raises(ValueError, fn, a, axis=-4)


def test_max():
    _ext_common(ht.max, torch.max, np.max, lambda p: p - 2)


def test_min():
    _ext_common(ht.min, torch.min, np.min, lambda p: 0)


def _pairwise_common(fn, npfn, tfn):
    d1 = [[1, 2, 3], [4, 5, 6], [7, 8, 9], [10, 11, 12]]
    d2 = [[0, 3, 2], [5, 4, 7], [6, 9, 8], [9, 10, 11]]
    r = fn(ht.array(d1), ht.array(d2))
    assert r.shape == (4, 3) and r.split is None and r.dtype == ht.int64
    assert torch.equal(r.larray.cpu(), tfn(torch.tensor(d1), torch.tensor(d2)))
    v1 = rng(24).standard_normal((6, 3, 3)).astype(np.float32)
    v2 = rng(25).standard_normal((6, 1, 3)).astype(np.float32)
    for s in (None, 0, 2):
        r = fn(ht.array(v1, split=s), ht.array(v2, split=s if s != 1 else None))
        assert r.shape == (6, 3, 3) and r.dtype == ht.float32 and r.split == s
        same(r, npfn(v1, v2))
    r = fn(ht.array(rng(26).standard_normal(1)), ht.array(v1, split=1))
    assert r.split == 1 and r.dtype == ht.float64
    r = fn(ht.array(v1, split=0), ht.array(np.float32([0.5])))
    assert r.split == 0
    same(r, npfn(v1, np.float32(0.5)))
    r = fn(5, ht.array(v1, split=1))
    assert r.split == 1 and r.dtype == ht.float32
    same(r, npfn(5, v1))
    r = fn(ht.array(v1, split=1), 5.0)
    assert r.split == 1 and r.dtype == ht.float32
    out = ht.empty((6, 3, 3), split=0, dtype=ht.float32)
    fn(ht.array(v1, split=0), ht.array(v2, split=0), out=out)
    same(out, npfn(v1, v2))
    a1, a2 = ht.array(v1, split=0), ht.array(v2, split=0)
    raises(ValueError, fn, a1, ht.array([]))
    raises(ValueError, fn, a1, ht.array(rng(27).standard_normal((4, 2, 3)), split=0))
    # deliberate extensions (documented in core/_operations.py): torch/NumPy operands are promoted
    # to replicated arrays, and operands split along different axes are aligned with one
    # all-to-all, where the reference raises TypeError / NotImplementedError
    raises(ValueError, fn, a1, torch.ones(12, 3, 3))
    same(fn(a1, torch.ones(6, 3, 3)), npfn(v1, np.ones((6, 3, 3), np.float32)))
    same(fn(a1, ht.array(v1 * 0.5, split=1)), npfn(v1, v1 * 0.5))
    raises(TypeError, fn, a1, a2, out=torch.ones(12, 3, 3))
    raises(ValueError, fn, a1, a2, out=ht.ones((12, 4, 3)))
    raises(ValueError, fn, a1, a2, out=ht.ones((6, 3, 3), split=1))


def test_maximum():
    _pairwise_common(ht.maximum, np.maximum, torch.max)


def test_minimum():
    _pairwise_common(ht.minimum, np.minimum, torch.min)
    same(ht.minimum(np.array(7.2), ht.ones((2, 2))), np.ones((2, 2)))


def test_mean():
    x = ht.zeros((2, 3, 4))
    raises(ValueError, x.mean, axis=10)
    raises(ValueError, x.mean, axis=[4])
    raises(ValueError, x.mean, axis=[-4])
    raises(TypeError, ht.mean, x, axis="01")
    raises(ValueError, ht.mean, x, axis=(0, "10"))
    raises(ValueError, ht.mean, x, axis=(0, 0))
    raises(ValueError, ht.mean, x, axis=torch.Tensor([0, 0]))
    assert float(ht.arange(1, 5).mean()) == 2.5
    _ones_reductions(lambda z, **kw: z.mean(**kw), 1, 5)
    x = rng(28).standard_normal((5, 6, 7))
    for s in splits(3):
        h = ht.array(x, split=s)
        for ax in (None, 0, 1, 2, (0, 1), (1, 2), (0, 2)):
            close(ht.mean(h, axis=ax), np.mean(x, axis=ax), rtol=1e-10, atol=1e-12)
    for sp in (None, 0, 1):
        iris = _iris(sp)
        if iris is not None:
            assert ht.allclose(ht.mean(iris), 3.46366666666667)
            assert ht.allclose(ht.mean(iris, axis=0), ht.array([5.84333333333333, 3.054, 3.75866666666667,
                                                                 1.19866666666667]))


def _ones_reductions(fn, expect, n):
    dims = []
    for d in (n, n, n):
        dims.append(d)
        for split in list(range(len(dims))) + [None]:
            z = ht.ones(dims, split=split)
            assert ht.allclose(fn(z), expect)
            for it in range(len(dims)):
                res = fn(z, axis=it)
                assert ht.allclose(res, expect)
                assert res.gshape == tuple(d for q, d in enumerate(dims) if q != it)
                assert res.split == _split_after(z.split, it)
            for comb in combinations(range(len(dims)), 2):
                res = fn(z, axis=list(comb))
                assert ht.allclose(res, expect)
                target = tuple(d for q, d in enumerate(dims) if q not in comb)
                if res.gshape:
                    assert res.gshape == target
                if res.split is not None:
                    if any(split >= c for c in comb):
                        assert res.split == len(target) - 1
                    else:
                        assert res.split == z.split


def test_percentile():
    x_np = np.arange(3 * 10 * 10).reshape(3, 10, 10)
    hs = [ht.array(x_np, split=s) for s in splits(3)]
    q = 15.9
    for dim in range(3):
        p = np.percentile(x_np, q, axis=dim)
        for h in hs:
            close(ht.percentile(h, q, axis=dim), p, rtol=1e-12, atol=1e-9)
    for h in hs:
        close(ht.percentile(h, 100, axis=0), np.percentile(x_np, 100, axis=0))
        close(ht.median(h, axis=0), np.percentile(x_np, 50, axis=0))
    ql = [0.1, 2.3, 15.9, 50.0, 84.1, 97.7, 99.9]
    for h in hs:
        p_np = np.percentile(x_np, ql, axis=2, method="lower", keepdims=True)
        p = ht.percentile(h, ql, axis=2, interpolation="lower", keepdim=True)
        assert p.shape == p_np.shape
        close(p, p_np)
        out = ht.empty(p_np.shape, dtype=ht.float64, split=p.split)
        ht.percentile(h, ql, axis=2, out=out, interpolation="lower", keepdim=True)
        close(out, p_np)
        for m in ("higher", "nearest", "midpoint", "linear"):
            close(ht.percentile(h, ql, axis=None, interpolation=m), np.percentile(x_np, ql, method=m))
    q_ht = ht.array(ql, split=0)
    close(ht.percentile(hs[0], q_ht, interpolation="midpoint"), np.percentile(x_np, ql, method="midpoint"))
    close(ht.percentile(ht.array(4.5), q=ql), np.percentile(4.5, ql))
    h = hs[0]
    raises(TypeError, ht.percentile, x_np, ql)
    raises(ValueError, ht.percentile, h, ql, interpolation="Homer!")
    raises(NotImplementedError, ht.percentile, h, ql, axis=(0, 1))
    raises(TypeError, ht.percentile, h, np.array(ql))
    raises(TypeError, ht.percentile, h, ql, out=torch.empty((len(ql),), dtype=torch.float64))
    raises(TypeError, ht.percentile, h, ql, out=ht.empty((len(ql),), dtype=ht.float32))
    raises(ValueError, ht.percentile, h, ql, out=ht.empty((len(ql) + 1,), dtype=ht.float64))
    raises(ValueError, ht.percentile, h, ql, out=ht.empty((len(ql),), dtype=ht.float64, split=0))


def test_std():
    a = ht.arange(1, 5)
    assert abs(float(a.std()) - 1.118034) < 1e-6
    assert abs(float(a.std(bessel=True)) - 1.2909944) < 1e-6
    x = ht.zeros((2, 3, 4))
    raises(TypeError, ht.std, x, axis=0, ddof=1.0)
    raises(ValueError, ht.std, x, axis=10)
    raises(TypeError, ht.std, x, axis="01")
    raises(ValueError, ht.std, x, ddof=-2)
    d = rng(29).standard_normal((7, 5, 3))
    for s in splits(3):
        for ax in (None, 0, 1, 2):
            for dd in (0, 1):
                close(ht.std(ht.array(d, split=s), axis=ax, ddof=dd), np.std(d, axis=ax, ddof=dd), rtol=1e-10)


def test_var():
    x = ht.zeros((2, 3, 4))
    raises(ValueError, x.var, axis=10)
    raises(ValueError, x.var, axis=[4])
    raises(ValueError, x.var, axis=[-4])
    raises(TypeError, ht.var, x, axis="01")
    raises(TypeError, ht.var, x, ddof="01")
    raises(ValueError, ht.var, x, axis=(0, "10"))
    raises(ValueError, ht.var, x, axis=(0, 0))
    raises(NotImplementedError, ht.var, x, ddof=2)
    raises(ValueError, ht.var, x, ddof=-2)
    raises(ValueError, ht.var, x, axis=torch.Tensor([0, 0]))
    assert abs(float(ht.arange(1, 5).var(ddof=1)) - 1.666666666666666) < 1e-6
    _ones_reductions(lambda z, **kw: z.var(ddof=0, **kw), 0, ht.MPI_WORLD.size * 2)
    d = rng(30).standard_normal((9, 4, 3))
    for s in splits(3):
        for ax in (None, 0, 1, 2, (0, 2)):
            close(ht.var(ht.array(d, split=s), axis=ax, ddof=1), np.var(d, axis=ax, ddof=1), rtol=1e-10)
    for sp in (None, 0, 1):
        iris = _iris(sp)
        if iris is not None:
            assert ht.allclose(ht.var(iris, bessel=True), 3.90318519755147)
