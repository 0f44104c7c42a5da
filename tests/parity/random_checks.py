"""Parity with ``heat/core/tests/test_random.py``: the counter-based (Threefry) streams are
independent of split and shape (global element order), seed/set_state/get_state semantics
including counter overflow at 2^64 and 2^128, distribution sanity, the aliases, permutation/
randperm/randint/normal and the errors. (Bit-level equality with the reference's own streams is
parity-unpinned: the reference holds no fixture values.)"""
import numpy as np
import torch

import heat_amd as ht

from ._util import raises, same, splits


def test_rand():
    seed = 12345
    ht.random.seed(seed)
    a = ht.random.rand(2, 5, 7, 3, split=0)
    assert a.dtype == ht.float32 and a.larray.dtype == torch.float32
    b = ht.random.rand(2, 5, 7, 3, split=0)
    assert not ht.equal(a, b)
    ht.random.seed(seed)
    c = ht.random.rand(2, 5, 7, 3, dtype=ht.float32, split=0)
    assert ht.equal(a, c)
    # counter overflow past 2^64 continues the stream
    ht.random.set_state(("Threefry", seed, 0xFFFFFFFFFFFFFFF0))
    a = ht.random.rand(2, 3, 4, 5, split=0).numpy().flatten()
    ht.random.set_state(("Threefry", seed, 0x10000000000000000))
    b = ht.random.rand(2, 44, split=0).numpy().flatten()
    assert a.dtype == np.float32 and np.array_equal(a[32:], b)
    ht.random.set_state(("Threefry", seed, 0x100000000))
    a = ht.random.rand(2, 44)
    ht.random.seed(seed)
    assert not ht.equal(a, ht.random.rand(2, 44))
    # 128-bit wrap-around restarts the stream
    ht.random.seed(seed)
    a = ht.random.rand(2, 34, split=0).numpy().flatten()
    ht.random.set_state(("Threefry", seed, 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF0))
    b = ht.random.rand(2, 50, split=0).numpy().flatten()
    assert np.array_equal(a, b[32:])
    ht.random.seed(seed)
    a = ht.random.rand(3, 5, 2, 9, split=3)
    ht.random.seed(seed)
    assert ht.equal(a, ht.random.rand(3, 5, 2, 9, split=3))
    # split 0 and replicated arrays take the stream in global C order (split > 0: each rank one
    # contiguous piece of the stream, so only the value set agrees, like the reference)
    for s in (None, 0):
        ht.random.seed(seed)
        a = ht.random.rand(2, 50, split=s).numpy().flatten()
        ht.random.seed(seed)
        b = ht.random.rand(100, split=None).numpy()
        assert np.array_equal(a, b)
    ht.random.seed(seed)
    a = np.sort(ht.random.rand(3, 5, 2, 9, split=3).numpy().flatten())
    ht.random.seed(seed)
    b = np.sort(ht.random.rand(30, 9, split=1).numpy().flatten())
    assert np.array_equal(a, b)
    a = ht.random.rand(11, 15, 3, 7, split=2).numpy()
    assert (np.unique(a, return_counts=True)[1] == 1).all()
    b = ht.random.rand(14, 7, 3, 12, 18, 4, split=5, dtype=ht.float64)
    c = np.concatenate((a.flatten(), b.numpy().flatten()))
    assert (np.unique(c, return_counts=True)[1] == 1).all()
    assert 0.49 < np.mean(c) < 0.51 and 0.49 < np.median(c) < 0.51 and np.std(c) < 0.3
    assert ((0 <= c) & (c < 1)).all()
    ht.random.seed(seed)
    a = ht.random.rand()
    ht.random.seed(seed)
    b = ht.random.rand(1)
    assert float(a.item()) == float(b.item())
    raises(ValueError, ht.random.randn, 0x7FFFFFFFFFFFFFFF)
    raises(ValueError, ht.random.rand, 3, 2, -2, 5, split=1)
    raises(ValueError, ht.random.randn, 12, 43, dtype=ht.int32, split=0)


def test_randn():
    ht.random.seed(54321)
    for s in splits(3):
        a = ht.random.randn(30, 20, 10, split=s)
        assert a.dtype == ht.float32 and a.gshape == (30, 20, 10) and a.split == s
        v = a.numpy()
        assert abs(v.mean()) < 0.02 and abs(v.std() - 1) < 0.02
    ht.random.seed(7)
    a = ht.random.randn(4, 25, split=0).numpy().flatten()
    ht.random.seed(7)
    b = ht.random.randn(100).numpy()
    assert np.array_equal(a, b)
    a = ht.random.randn(10, 10, dtype=ht.float64, split=1)
    assert a.dtype == ht.float64


def test_standard_normal():
    ht.random.seed(3)
    a = ht.random.standard_normal((7, 5), split=0)
    ht.random.seed(3)
    b = ht.random.randn(7, 5, split=0)
    assert ht.equal(a, b)
    assert ht.random.standard_normal().shape == (1,)


def test_normal():
    shape = (3, 4, 6)
    ht.random.seed(2)
    g = ht.random.normal(shape=shape, split=2)
    ht.random.seed(2)
    assert ht.equal(g, ht.random.randn(*shape, split=2))
    mu = ht.array(np.arange(72.0).reshape(shape), split=2)
    ht.random.seed(22)
    g = ht.random.normal(mu, 2.0, shape, split=2)
    ht.random.seed(22)
    r = ht.random.randn(*shape, split=2)
    assert np.allclose(g.numpy(), mu.numpy() + 2.0 * r.numpy(), atol=1e-4)
    raises(TypeError, ht.random.normal, [4, 5], 1, shape)
    raises(TypeError, ht.random.normal, 0, "r", shape)
    raises(ValueError, ht.random.normal, 0, -1, shape)


def test_randint():
    ht.random.seed(13579)
    for s in splits(2):
        a = ht.random.randint(3, 17, size=(30, 40), split=s)
        assert a.dtype == ht.int32 and a.split == s
        v = a.numpy()
        assert v.min() >= 3 and v.max() < 17 and len(np.unique(v)) == 14
    a = ht.random.randint(10, size=(5,), dtype=ht.int64)
    assert a.dtype == ht.int64 and (a.numpy() < 10).all()
    ht.random.seed(5)
    a = ht.random.randint(0, 1000, size=(4, 25), split=0).numpy().flatten()
    ht.random.seed(5)
    assert np.array_equal(a, ht.random.randint(0, 1000, size=(100,)).numpy())
    v = ht.random.randint(0, 10000, size=(100000,), split=0).numpy()
    assert 4900 < v.mean() < 5100 and v.std() < 2900
    raises(ValueError, ht.random.randint, 5, 5, size=(10, 10), split=0)
    raises(ValueError, ht.random.randint, low=0, high=10, size=(3, -4))
    raises(ValueError, ht.random.randint, low=0, high=10, size=(15,), dtype=ht.float32)


def test_randperm():
    ht.random.seed(8)
    for s in (None, 0):
        p = ht.random.randperm(25, split=s)
        assert p.dtype == ht.int64 and p.split == s
        assert np.array_equal(np.sort(p.numpy()), np.arange(25))
    p = ht.random.randperm(10, dtype=ht.int32)
    assert p.dtype == ht.int32
    ht.random.seed(8)
    a = ht.random.randperm(40, split=0).numpy()
    ht.random.seed(8)
    assert np.array_equal(a, ht.random.randperm(40).numpy())
    raises(TypeError, ht.random.randperm, "abc")


def test_permutation():
    ht.random.seed()
    a = ht.random.permutation(10)
    assert np.array_equal(np.sort(a.numpy()), np.arange(10))
    x = np.arange(60.0).reshape(12, 5)
    for s in splits(2):
        p = ht.random.permutation(ht.array(x, split=s))
        assert p.gshape == x.shape and (p.split == s or s == 1)
        got = p.numpy()
        # rows are permuted whole
        assert np.array_equal(np.sort(got[:, 0]), x[:, 0])
        for row in got:
            assert np.array_equal(row, x[int(row[0]) // 5])
    raises(TypeError, ht.random.permutation, "abc")


def test_random_sample():
    ht.random.seed(534)
    a = ht.random.rand(6, 2, 3)
    for fn in (ht.random.random, ht.random.random_sample, ht.random.ranf, ht.random.sample):
        ht.random.seed(534)
        assert ht.equal(a, fn((6, 2, 3)))
    assert ht.random.random_sample().shape == (1,)


def test_set_state():
    ht.random.set_state(("Threefry", 12345, 0xFFF))
    assert ht.random.get_state() == ("Threefry", 12345, 0xFFF, 0, 0.0)
    ht.random.set_state(("Threefry", 55555, 0xFFFFFFFFFFFFFF, "for", "compatibility"))
    assert ht.random.get_state() == ("Threefry", 55555, 0xFFFFFFFFFFFFFF, 0, 0.0)
    raises(ValueError, ht.random.set_state, ("Thrfry", 12, 0xF))
    raises(TypeError, ht.random.set_state, ("Threefry", 12345))
