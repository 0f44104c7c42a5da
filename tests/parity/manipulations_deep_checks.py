"""Deeper parity with ``heat/core/tests/test_manipulations.py``: the same manipulations on
UNBALANCED inputs (skewed lshape maps with empty ranks, the layouts slicing and redistribution
leave behind - the reference tests build them with ``redistribute_``), mixed-dtype promotion,
output split rules, empty arrays and the reference's error cases (``test_manipulations.py``
assertRaises blocks, e.g. lines 348-364, 420-431, 697-706, 897-903, 1466-1489, 1800-1835,
2310-2322, 2506-2563, 2840-2852, 3170-3176, 3235-3267)."""
import numpy as np
import torch

import heat_amd as ht

from ._util import raises, rng, same, splits


def _skewed(data, split, dtype=None):
    """``data`` distributed along ``split`` with a skewed layout: rank 0 holds half of the split
    axis, odd ranks nothing, the rest spread over the remaining even ranks."""
    x = ht.array(data, split=split, dtype=dtype)
    if split is None or x.comm.size == 1:
        return x
    p, n = x.comm.size, data.shape[split]
    counts = [0] * p
    counts[0] = n // 2
    rest = n - counts[0]
    evens = [r for r in range(2, p, 2)] or [0]
    for i in range(rest):
        counts[evens[i % len(evens)]] += 1
    target = x.create_lshape_map().clone()
    target[:, split] = torch.tensor(counts)
    x.redistribute_(lshape_map=x.create_lshape_map(), target_map=target)
    assert x.lshape[split] == counts[x.comm.rank]
    return x


A3 = rng(1).standard_normal((9, 7, 5)).astype(np.float32)
A2 = rng(2).standard_normal((11, 6)).astype(np.float32)
V1 = rng(3).standard_normal(13).astype(np.float32)


def test_concatenate_unbalanced_and_promotion():
    for s in splits(3):
        for ax in range(3):
            other = np.take(A3, range(3), axis=ax) * 2
            got = ht.concatenate((_skewed(A3, s), _skewed(other, s)), axis=ax)
            same(got, np.concatenate((A3, other), axis=ax))
            assert got.split == s
    # dtype promotion int + float like the reference (test_manipulations.py:300-340)
    i = np.arange(12, dtype=np.int32).reshape(4, 3)
    f = np.ones((2, 3), dtype=np.float64)
    r = ht.concatenate((ht.array(i, split=0), ht.array(f, split=0)))
    assert r.dtype == ht.float64
    same(r, np.concatenate((i, f)))
    # split + None: the result keeps the split
    r = ht.concatenate((ht.array(A2, split=0), ht.array(A2, split=None)), axis=0)
    assert r.split == 0
    same(r, np.concatenate((A2, A2)))
    r = ht.concatenate((ht.array(A2, split=None), ht.array(A2, split=1)), axis=0)
    assert r.split == 1
    same(r, np.concatenate((A2, A2)))
    raises(ValueError, ht.concatenate, (ht.zeros((6, 3, 5)), ht.zeros((4, 5, 1))))
    raises(TypeError, ht.concatenate, (ht.zeros((6, 3, 5)), "ab"))
    raises(TypeError, ht.concatenate, (ht.zeros((6, 3, 5)), ht.zeros((6, 3, 5))), axis="0")
    raises(RuntimeError, ht.concatenate, (ht.zeros((6, 3, 5), split=0), ht.zeros((6, 3, 5), split=1)))


def test_concatenate_empty_blocks():
    e = np.zeros((0, 4), dtype=np.float32)
    d = np.arange(8, dtype=np.float32).reshape(2, 4)
    for s in (None, 0, 1):
        same(ht.concatenate((ht.array(e, split=s), ht.array(d, split=s))), np.concatenate((e, d)))
        same(ht.concatenate((ht.array(d, split=s), ht.array(e, split=s))), np.concatenate((d, e)))


def test_diag_unbalanced():
    for s in (None, 0):
        for k in (-4, 0, 2):
            same(ht.diag(_skewed(V1, s), offset=k), np.diag(V1, k))
    for s in splits(2):
        for k in (-3, 0, 4):
            same(ht.diag(_skewed(A2, s), offset=k), np.diag(A2, k))
    raises(TypeError, ht.diag, A2)
    raises(ValueError, ht.diag, ht.array(V1), offset=None)
    raises(ValueError, ht.diag, ht.array(V1), offset="3")
    raises(ValueError, ht.diag, ht.empty([]))
    same(ht.diag(ht.array(A3, split=0)), np.diagonal(A3))   # > 2-D: the diagonal (reference)


def test_diagonal_unbalanced_and_errors():
    for s in splits(3):
        x = _skewed(A3, s)
        for d1, d2 in ((0, 1), (1, 2), (0, 2), (2, 0)):
            for k in (-2, 0, 3):
                same(ht.diagonal(x, offset=k, dim1=d1, dim2=d2), np.diagonal(A3, k, axis1=d1, axis2=d2))
    raises(ValueError, ht.diagonal, ht.array(A2), offset=None)
    raises(ValueError, ht.diagonal, ht.array(np.arange(3.0)))


def test_expand_dims_split_shift():
    for s in splits(3):
        for ax in (0, 1, 2, 3, -1, -4):
            r = ht.expand_dims(_skewed(A3, s), ax)
            same(r, np.expand_dims(A3, ax))
            if s is not None:
                a = ax % 4
                assert r.split == (s + 1 if a <= s else s)
    raises(TypeError, ht.expand_dims, "(3, 4, 5,)", 1)
    raises(TypeError, ht.expand_dims, ht.array(A3), "1")
    raises(ValueError, ht.expand_dims, ht.array(A3), 4)
    raises(ValueError, ht.expand_dims, ht.array(A3), -5)


def test_flatten_ravel_unbalanced():
    for s in splits(3):
        x = _skewed(A3, s)
        same(ht.flatten(x), A3.ravel())
        same(ht.ravel(x), A3.ravel())
        assert ht.flatten(x).split == (None if s is None else 0)
    e = ht.array(np.zeros((0, 3), np.float32), split=0)
    assert ht.flatten(e).shape == (0,)


def test_flip_unbalanced():
    for s in splits(3):
        x = _skewed(A3, s)
        for ax in (None, 0, 1, 2, (0, 1), (1, 2), (0, 1, 2), -1):
            r = ht.flip(x, ax)
            same(r, np.flip(A3, ax))
            assert r.split == s
        same(ht.flipud(x), np.flipud(A3))
    for s in splits(2):
        same(ht.fliplr(_skewed(A2, s)), np.fliplr(A2))


def test_moveaxis_swapaxes_errors():
    for s in splits(3):
        x = _skewed(A3, s)
        same(ht.moveaxis(x, -1, 0), np.moveaxis(A3, -1, 0))
        same(ht.moveaxis(x, (0, 2), (1, 0)), np.moveaxis(A3, (0, 2), (1, 0)))
        same(ht.swapaxes(x, 1, -1), np.swapaxes(A3, 1, -1))
    raises(TypeError, ht.moveaxis, ht.array(A3), source="r", destination=3)
    raises(TypeError, ht.moveaxis, ht.array(A3), source=2, destination=3.0)
    raises(ValueError, ht.moveaxis, ht.array(A3), source=(0, 0), destination=(1, 2))
    raises(ValueError, ht.moveaxis, ht.array(A3), source=(0, 1), destination=(2,))
    raises((ValueError, IndexError), ht.swapaxes, ht.array(A3), 0, 3)


def test_pad_unbalanced_and_errors():
    for s in splits(3):
        x = _skewed(A3, s)
        same(ht.pad(x, ((1, 0), (0, 2), (3, 1))), np.pad(A3, ((1, 0), (0, 2), (3, 1))))
        same(ht.pad(x, 1, constant_values=-2), np.pad(A3, 1, constant_values=-2))
        same(ht.pad(x, ((2, 2),)), np.pad(A3, ((2, 2),)))
    for s in splits(2):
        same(ht.pad(_skewed(A2, s), [(0, 3), (1, 1)], constant_values=((1, 2), (3, 4))),
             np.pad(A2, [(0, 3), (1, 1)], constant_values=((1, 2), (3, 4))))
    raises(TypeError, ht.pad, "[[3, 4, 5],[6,7,8]]", 3)
    raises(TypeError, ht.pad, ht.array(A2), "(1, 1)")
    raises(ValueError, ht.pad, ht.array(A2), ((1, 2), (1, 2), (1, 2)))
    raises(ValueError, ht.pad, ht.array(A2), ((1, 2, 3), (1, 2)))


def test_repeat_unbalanced_and_errors():
    for s in (None, 0):
        x = _skewed(V1, s)
        same(ht.repeat(x, 2), np.repeat(V1, 2))
        reps = np.arange(13) % 3
        same(ht.repeat(x, reps), np.repeat(V1, reps))
        same(ht.repeat(x, ht.array(reps)), np.repeat(V1, reps))
    for s in splits(2):
        x = _skewed(A2, s)
        same(ht.repeat(x, 3, axis=0), np.repeat(A2, 3, axis=0))
        same(ht.repeat(x, [1, 2, 0, 1, 3, 1], axis=1), np.repeat(A2, [1, 2, 0, 1, 3, 1], axis=1))
    raises(TypeError, ht.repeat, ht.array(A2), 2, axis="0")
    raises(TypeError, ht.repeat, ht.array(A2), 2.5)
    raises(ValueError, ht.repeat, ht.array(A2), [1, 2], axis=0)
    raises(ValueError, ht.repeat, ht.array(A2), 2, axis=2)


def test_reshape_unbalanced_new_split():
    for s in splits(3):
        x = _skewed(A3, s)
        for shp in ((315,), (21, 15), (3, 3, 35), (5, 7, 9), (-1, 5)):
            for ns in [None] + list(range(len(shp))):
                r = ht.reshape(x, shp, new_split=ns)
                same(r, A3.reshape(shp))
                if ns is not None:
                    assert r.split == ns
    raises(ValueError, ht.reshape, ht.zeros((4, 3)), (5, 7))
    raises(ValueError, ht.reshape, ht.zeros((4, 3)), (-1, -1))
    raises(TypeError, ht.reshape, ht.zeros((4, 3)), "12")


def test_roll_unbalanced():
    for s in splits(3):
        x = _skewed(A3, s)
        for shift, ax in ((4, None), (-11, None), (3, 0), (-2, 1), (7, 2), ((1, -3), (0, 2)), ((2, 2), (1, 1))):
            same(ht.roll(x, shift, ax), np.roll(A3, shift, ax))
    raises(TypeError, ht.roll, ht.array(A3), 1.0, 0)
    raises(TypeError, ht.roll, ht.array(A3), 1, 1.0)
    raises(ValueError, ht.roll, ht.array(A3), (1, 2), (0, 1, 2))


def test_rot90_errors():
    for s in splits(3):
        x = _skewed(A3, s)
        for k in (1, 2, 3, -2):
            for axes in ((0, 1), (1, 2), (2, 0)):
                same(ht.rot90(x, k, axes), np.rot90(A3, k, axes))
    raises(ValueError, ht.rot90, ht.ones((2, 3)), 1, (0, 1, 2))
    raises(ValueError, ht.rot90, ht.ones((2, 3)), 1, (0, 5))
    raises(TypeError, ht.rot90, ht.ones((2, 3)), 1.5)
    raises(TypeError, ht.rot90, "[[1, 2], [3, 4]]")


def test_sort_unbalanced_and_out():
    d = rng(7).standard_normal((17, 6)).astype(np.float32)
    d[3, 2] = d[5, 2]   # a tie
    for s in splits(2):
        x = _skewed(d, s)
        for ax in (0, 1, -1):
            v, i = ht.sort(x, axis=ax)
            same(v, np.sort(d, axis=ax))
            same(np.take_along_axis(d, i.numpy(), ax), np.sort(d, axis=ax))
            assert v.split == s
    out = ht.empty((17, 6), split=0)
    ht.sort(ht.array(d, split=0), axis=0, out=out)
    same(out, np.sort(d, axis=0))
    ints = rng(8).integers(-50, 50, 40).astype(np.int64)
    v, _ = ht.sort(_skewed(ints, 0), descending=True)
    same(v, np.sort(ints)[::-1])
    raises(ValueError, ht.sort, ht.array(d), axis=2)
    raises(TypeError, ht.sort, ht.array(d), axis="1")


def test_split_family_errors():
    for s in splits(3):
        x = _skewed(A3, s)
        for g, e in zip(ht.split(x, [2, 5, 7], axis=0), np.split(A3, [2, 5, 7], axis=0)):
            same(g, e)
        for g, e in zip(ht.split(x, ht.array([1, 3]), axis=2), np.split(A3, [1, 3], axis=2)):
            same(g, e)
        for g, e in zip(ht.split(x, 7, axis=1), np.split(A3, 7, axis=1)):
            same(g, e)
    raises(TypeError, ht.split, [1, 2, 3, 4], 2)
    raises(TypeError, ht.split, ht.array(A3), 1.5)
    raises(ValueError, ht.split, ht.array(A3), 2, axis=0)
    raises(ValueError, ht.split, ht.array(A3), 1, axis=3)
    raises(ValueError, ht.vsplit, ht.array(V1), 1)


def test_squeeze_errors():
    d = np.arange(12.0, dtype=np.float32).reshape(1, 4, 1, 3, 1)
    for s in splits(5):
        x = _skewed(d, s)
        same(ht.squeeze(x), np.squeeze(d))
        same(ht.squeeze(x, (0, 4)), np.squeeze(d, (0, 4)))
        same(ht.squeeze(x, -3), np.squeeze(d, -3))
    raises(TypeError, ht.squeeze, ht.array(d), axis=1.1)
    raises(TypeError, ht.squeeze, ht.array(d), axis="0")
    raises(ValueError, ht.squeeze, ht.array(d), axis=1)
    raises(ValueError, ht.squeeze, ht.array(d), axis=(0, 1))


def test_stack_splits_and_errors():
    b = A2 * 3
    for s in splits(2):
        for ax in (0, 1, 2, -1, -3):
            r = ht.stack((_skewed(A2, s), ht.array(b, split=s)), axis=ax)
            same(r, np.stack((A2, b), axis=ax))
            if s is not None:
                a = ax % 3
                assert r.split == (s + 1 if a <= s else s)
    out = ht.empty((2, 11, 6), split=1)
    ht.stack((ht.array(A2, split=0), ht.array(b, split=0)), out=out)
    same(out, np.stack((A2, b)))
    raises(TypeError, ht.stack, (ht.array(A2), A2, ht.array(b)))
    raises(TypeError, ht.stack, ht.array(A2))
    raises(ValueError, ht.stack, (ht.array(A2),))
    raises(ValueError, ht.stack, (ht.array(A2), ht.array(A2.T)))
    raises(ValueError, ht.stack, (ht.array(A2, split=0), ht.array(A2, split=1)))


def test_hvstack_column_row_stack_unbalanced():
    c = np.arange(11.0, dtype=np.float32)
    for s in (None, 0):
        same(ht.column_stack((_skewed(A2, s), ht.array(c, split=s))), np.column_stack((A2, c)))
        same(ht.vstack((_skewed(A2, s), ht.array(A2[:2], split=s))), np.vstack((A2, A2[:2])))
        same(ht.row_stack((_skewed(V1[:6], s), ht.array(A2, split=s))), np.vstack((V1[:6], A2)))
        same(ht.hstack((_skewed(A2, s), ht.array(A2[:, :1], split=s))), np.hstack((A2, A2[:, :1])))
    raises(ValueError, ht.column_stack, (ht.array(A2), ht.array(np.arange(4.0))))
    raises(ValueError, ht.vstack, (ht.array(A2), ht.array(np.arange(4.0))))


def test_tile_unbalanced_and_errors():
    for s in splits(3):
        x = _skewed(A3, s)
        for reps in (2, (1, 2), (2, 1, 3), (2, 1, 1, 2), (0, 1, 2)):
            same(ht.tile(x, reps), np.tile(A3, reps))
    raises(TypeError, ht.tile, ht.array(A3), (1, 2, 2, 1.5))
    raises(TypeError, ht.tile, ht.array(A3), "12")
    raises(TypeError, ht.tile, A3, 2)


def test_topk_unbalanced():
    d = rng(9).standard_normal((12, 9)).astype(np.float32)
    for s in splits(2):
        x = _skewed(d, s)
        for dim in (0, 1):
            for k in (1, 4):
                v, i = ht.topk(x, k, dim=dim, largest=False)
                tv, _ = torch.topk(torch.tensor(d), k, dim=dim, largest=False)
                same(v, tv.numpy())
                same(np.take_along_axis(d, i.numpy(), dim), tv.numpy())
    out = (ht.empty((2, 9), split=None), ht.empty((2, 9), dtype=ht.int64, split=None))
    ht.topk(ht.array(d, split=0), 2, dim=0, out=out)
    same(out[0], torch.topk(torch.tensor(d), 2, dim=0)[0].numpy())


def test_unique_unbalanced():
    d = rng(10).integers(0, 6, (14, 3)).astype(np.int64)
    for s in splits(2):
        x = _skewed(d, s)
        same(ht.unique(x, sorted=True), np.unique(d))
        u, inv = ht.unique(x, sorted=True, return_inverse=True)
        same(u.numpy()[inv.numpy()].reshape(d.shape), d)
        same(ht.unique(x, sorted=True, axis=0), np.unique(d, axis=0))
        same(ht.unique(x, sorted=True, axis=1), np.unique(d, axis=1))
    v = rng(11).integers(0, 4, 25).astype(np.float32)
    same(ht.unique(_skewed(v, 0), sorted=True), np.unique(v))


def test_resplit_unbalanced_roundtrip():
    for a in splits(3):
        x = _skewed(A3, a)
        for b in splits(3):
            y = ht.resplit(x, b)
            assert y.split == b and (b == a or y.is_balanced())   # same split: a copy (reference)
            same(y, A3)
            if b is not None:
                z = ht.resplit(y, a)
                same(z, A3)
    raises(TypeError, ht.resplit, ht.array(A3, split=0), "1")
    raises(ValueError, ht.resplit, ht.array(A3, split=0), 3)


def test_balance_redistribute_roundtrip():
    for s in splits(3):
        if s is None:
            continue
        x = _skewed(A3, s)
        assert x.comm.size == 1 or not x.is_balanced(force_check=True) or A3.shape[s] < x.comm.size
        x.balance_()
        assert x.is_balanced(force_check=True)
        same(x, A3)
