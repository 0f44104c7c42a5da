"""Parity with ``heat/core/tests/test_manipulations.py``: every manipulation against NumPy on
every split (including splits along the manipulated axis), output split rules and error cases."""
import numpy as np
import torch

import heat_amd as ht

from ._util import close, raises, rng, same, splits

D3 = np.arange(4 * 5 * 6).reshape(4, 5, 6).astype(np.float32)
D2 = np.arange(7 * 4).reshape(7, 4).astype(np.float32)


def _each(data, fn, npfn, **kw):
    for s in splits(data.ndim):
        same(fn(ht.array(data, split=s), **kw), npfn(data, **kw) if kw else npfn(data))


def test_column_stack():
    a, b = np.arange(5.0), np.arange(5.0, 10.0)
    c = np.arange(10.0).reshape(5, 2)
    for s in (None, 0):
        same(ht.column_stack((ht.array(a, split=s), ht.array(b, split=s))), np.column_stack((a, b)))
        same(ht.column_stack((ht.array(a, split=s), ht.array(c, split=s))), np.column_stack((a, c)))
    raises(ValueError, ht.column_stack, (ht.array(a), ht.array(np.arange(3.0))))


def test_concatenate():
    x, y = D3, D3[:, :2] * 10
    for s in splits(3):
        for ax in range(3):
            yy = np.concatenate([x] * 2, axis=ax) if ax != 1 else np.concatenate([x, y], axis=1)
            other = x if ax != 1 else y
            same(ht.concatenate((ht.array(x, split=s), ht.array(other, split=s)), axis=ax), yy)
    same(ht.concatenate((ht.array(D2, split=0), ht.array(D2, split=0), ht.array(D2, split=0))),
         np.concatenate([D2] * 3))
    raises(ValueError, ht.concatenate, (ht.array(D2), ht.array(D3)))
    raises(TypeError, ht.concatenate, "ab")
    raises(ValueError, ht.concatenate, (ht.array(D2),), axis=3)


def test_diag():
    v = np.arange(6.0)
    for s in (None, 0):
        for k in (-2, 0, 3):
            same(ht.diag(ht.array(v, split=s), offset=k), np.diag(v, k))
    for s in splits(2):
        for k in (-1, 0, 2):
            same(ht.diag(ht.array(D2, split=s), offset=k), np.diag(D2, k))


def test_diagonal():
    for s in splits(2):
        for k in (-3, 0, 1):
            same(ht.diagonal(ht.array(D2, split=s), offset=k), np.diagonal(D2, k))
    for s in splits(3):
        same(ht.diagonal(ht.array(D3, split=s), dim1=0, dim2=2), np.diagonal(D3, axis1=0, axis2=2))
    raises(ValueError, ht.diagonal, ht.array(D2), dim1=1, dim2=1)


def test_dsplit():
    for s in splits(3):
        for i, (g, e) in enumerate(zip(ht.dsplit(ht.array(D3, split=s), 3), np.dsplit(D3, 3))):
            same(g, e)
        for g, e in zip(ht.dsplit(ht.array(D3, split=s), [1, 4]), np.dsplit(D3, [1, 4])):
            same(g, e)
    raises(ValueError, ht.dsplit, ht.array(D2), 2)


def test_expand_dims():
    for s in splits(2):
        for ax in (0, 1, 2, -1):
            e = ht.expand_dims(ht.array(D2, split=s), ax)
            same(e, np.expand_dims(D2, ax))
    raises(ValueError, ht.expand_dims, ht.array(D2), 4)


def test_flatten():
    _each(D3, ht.flatten, np.ravel)


def test_flip():
    for s in splits(3):
        for ax in (None, 0, 1, (0, 2)):
            same(ht.flip(ht.array(D3, split=s), ax), np.flip(D3, ax))


def test_fliplr():
    _each(D2, ht.fliplr, np.fliplr)
    raises((IndexError, ValueError), ht.fliplr, ht.array(np.arange(3)))


def test_flipud():
    _each(D3, ht.flipud, np.flipud)


def test_hsplit():
    for s in splits(2):
        for g, e in zip(ht.hsplit(ht.array(D2, split=s), 2), np.hsplit(D2, 2)):
            same(g, e)
    v = np.arange(12.0)
    for g, e in zip(ht.hsplit(ht.array(v, split=0), [3, 7]), np.hsplit(v, [3, 7])):
        same(g, e)


def test_hstack():
    a, b = np.arange(6.0).reshape(3, 2), np.arange(9.0).reshape(3, 3)
    for s in splits(2):
        same(ht.hstack((ht.array(a, split=s), ht.array(b, split=s))), np.hstack((a, b)))
    same(ht.hstack((ht.array(np.arange(3.0), split=0), ht.array(np.arange(4.0), split=0))),
         np.hstack((np.arange(3.0), np.arange(4.0))))


def test_moveaxis():
    for s in splits(3):
        x = ht.array(D3, split=s)
        same(ht.moveaxis(x, 0, -1), np.moveaxis(D3, 0, -1))
        same(ht.moveaxis(x, [0, 1], [2, 0]), np.moveaxis(D3, [0, 1], [2, 0]))
    raises(ValueError, ht.moveaxis, ht.array(D3), [0, 1], [0])


def test_pad():
    for s in splits(2):
        x = ht.array(D2, split=s)
        same(ht.pad(x, 2), np.pad(D2, 2))
        same(ht.pad(x, ((1, 2), (3, 0)), constant_values=7), np.pad(D2, ((1, 2), (3, 0)), constant_values=7))
        same(ht.pad(x, (1, 3)), np.pad(D2, (1, 3)))
    raises(TypeError, ht.pad, ht.array(D2), "x")
    raises(ValueError, ht.pad, ht.array(D2), ((1, 2, 3),))


def test_ravel():
    _each(D3, ht.ravel, np.ravel)


def test_repeat():
    v = np.arange(5.0)
    for s in (None, 0):
        same(ht.repeat(ht.array(v, split=s), 3), np.repeat(v, 3))
        same(ht.repeat(ht.array(v, split=s), [1, 0, 2, 3, 1]), np.repeat(v, [1, 0, 2, 3, 1]))
    for s in splits(2):
        same(ht.repeat(ht.array(D2, split=s), 2, axis=1), np.repeat(D2, 2, axis=1))
        same(ht.repeat(ht.array(D2, split=s), 2), np.repeat(D2, 2))
    raises(TypeError, ht.repeat, ht.array(v), "3")


def test_reshape():
    for s in splits(3):
        x = ht.array(D3, split=s)
        for shp in ((120,), (6, 20), (2, 3, 4, 5), (-1, 12)):
            if s is not None and s >= len(shp):
                raises(ValueError, ht.reshape, x, shp)  # the split axis must exist (reference)
                same(ht.reshape(x, shp, new_split=0), D3.reshape(shp))
                continue
            same(ht.reshape(x, shp), D3.reshape(shp))
        if s != 2:
            same(x.reshape(10, 12), D3.reshape(10, 12))
    r = ht.reshape(ht.array(D3, split=1), (6, 20), new_split=1)
    assert r.split == 1
    same(r, D3.reshape(6, 20))
    raises(ValueError, ht.reshape, ht.array(D3), (7, 7))


def test_roll():
    for s in splits(3):
        x = ht.array(D3, split=s)
        same(ht.roll(x, 2), np.roll(D3, 2))
        same(ht.roll(x, -3, axis=1), np.roll(D3, -3, axis=1))
        same(ht.roll(x, (1, 2), axis=(0, 2)), np.roll(D3, (1, 2), axis=(0, 2)))
    raises(TypeError, ht.roll, ht.array(D3), 1.5)


def test_rot90():
    for s in splits(2):
        for k in (-1, 0, 1, 2, 3, 5):
            same(ht.rot90(ht.array(D2, split=s), k), np.rot90(D2, k))
    same(ht.rot90(ht.array(D3, split=2), 1, (0, 2)), np.rot90(D3, 1, (0, 2)))
    raises(ValueError, ht.rot90, ht.array(D2), 1, (0, 0))


def test_row_stack():
    a, b = np.arange(4.0), np.arange(4.0, 8.0)
    for s in (None, 0):
        same(ht.row_stack((ht.array(a, split=s), ht.array(b, split=s))), np.vstack((a, b)))
    same(ht.row_stack((ht.array(D2, split=0), ht.array(np.arange(4.0), split=0))), np.vstack((D2, np.arange(4.0))))


def test_shape():
    for s in splits(3):
        assert ht.shape(ht.array(D3, split=s)) == D3.shape
    raises(TypeError, ht.shape, D3)


def test_sort():
    d = rng(3).standard_normal((9, 5)).astype(np.float32)
    for s in splits(2):
        for ax in (0, 1):
            for desc in (False, True):
                v, i = ht.sort(ht.array(d, split=s), axis=ax, descending=desc)
                ref = np.sort(d, axis=ax)
                if desc:
                    ref = np.flip(ref, ax)
                same(v, ref)
                same(np.take_along_axis(d, i.numpy(), ax), ref)
    raises(ValueError, ht.sort, ht.array(d), axis=3)


def test_split():
    for s in splits(3):
        x = ht.array(D3, split=s)
        for ax in range(3):
            n = D3.shape[ax]
            for g, e in zip(ht.split(x, [1, n - 1], axis=ax), np.split(D3, [1, n - 1], axis=ax)):
                same(g, e)
        for g, e in zip(ht.split(x, 2), np.split(D3, 2)):
            same(g, e)
    raises(ValueError, ht.split, ht.array(D3), 3)


def test_resplit():
    for a in splits(3):
        for b in splits(3):
            y = ht.resplit(ht.array(D3, split=a), b)
            assert y.split == b
            same(y, D3)


def test_squeeze():
    d = np.arange(6.0).reshape(1, 3, 1, 2)
    for s in splits(4):
        same(ht.squeeze(ht.array(d, split=s)), np.squeeze(d))
        same(ht.squeeze(ht.array(d, split=s), 2), np.squeeze(d, 2))
    raises(ValueError, ht.squeeze, ht.array(d), 1)


def test_stack():
    for s in splits(2):
        for ax in (0, 1, 2, -1):
            same(ht.stack((ht.array(D2, split=s), ht.array(D2 + 1, split=s)), axis=ax),
                 np.stack((D2, D2 + 1), axis=ax))
    raises(ValueError, ht.stack, (ht.array(D2), ht.array(D3)))


def test_swapaxes():
    for s in splits(3):
        same(ht.swapaxes(ht.array(D3, split=s), 0, 2), np.swapaxes(D3, 0, 2))
    raises(TypeError, ht.swapaxes, ht.array(D3), "0", 1)


def test_tile():
    v = np.arange(4.0)
    for s in (None, 0):
        same(ht.tile(ht.array(v, split=s), 3), np.tile(v, 3))
        same(ht.tile(ht.array(v, split=s), (2, 2)), np.tile(v, (2, 2)))
    for s in splits(2):
        same(ht.tile(ht.array(D2, split=s), (2, 3)), np.tile(D2, (2, 3)))
        same(ht.tile(ht.array(D2, split=s), (2, 1, 2)), np.tile(D2, (2, 1, 2)))


def test_topk():
    d = rng(4).standard_normal((8, 11)).astype(np.float32)
    for s in splits(2):
        for dim in (0, 1):
            for largest in (True, False):
                v, i = ht.topk(ht.array(d, split=s), 3, dim=dim, largest=largest)
                tv, ti = torch.topk(torch.tensor(d), 3, dim=dim, largest=largest)
                same(v, tv.numpy())
                same(np.take_along_axis(d, i.numpy(), dim), tv.numpy())


def test_unique():
    d = np.array([[3, 1, 3], [2, 1, 4], [3, 0, 2]], dtype=np.int32)
    for s in splits(2):
        same(ht.unique(ht.array(d, split=s), sorted=True), np.unique(d))
        u, inv = ht.unique(ht.array(d, split=s), sorted=True, return_inverse=True)
        same(u.numpy()[inv.numpy()].reshape(d.shape) if inv.ndim == 2 else u.numpy()[inv.numpy()],
             d if inv.ndim == 2 else d.reshape(-1))
        same(ht.unique(ht.array(d, split=s), sorted=True, axis=0), np.unique(d, axis=0))


def test_vsplit():
    for s in splits(2):
        d = np.arange(8 * 3.0).reshape(8, 3)
        for g, e in zip(ht.vsplit(ht.array(d, split=s), 4), np.vsplit(d, 4)):
            same(g, e)
        for g, e in zip(ht.vsplit(ht.array(d, split=s), [2, 5]), np.vsplit(d, [2, 5])):
            same(g, e)


def test_vstack():
    for s in splits(2):
        same(ht.vstack((ht.array(D2, split=s), ht.array(D2 * 2, split=s))), np.vstack((D2, D2 * 2)))
    same(ht.vstack((ht.array(np.arange(3.0), split=0), ht.array(np.arange(3.0), split=0))),
         np.vstack((np.arange(3.0), np.arange(3.0))))
