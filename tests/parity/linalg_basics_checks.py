"""Parity with ``heat/core/linalg/tests/test_basics.py``: dot/matmul over every split pairing
(and batched), matrix/vector/general norms, outer (output split rules, out= buffers), projection,
trace (2-D and n-D, offsets, axes), transpose, tril/triu and vecdot against NumPy, with the
reference's errors."""
import numpy as np
import torch

import heat_amd as ht

from ._util import close, raises, rng, same, splits


def test_dot():
    a1, b1 = rng(1).standard_normal(11), rng(2).standard_normal(11)
    for s in (None, 0):
        for t in (None, 0):
            r = ht.dot(ht.array(a1, split=s), ht.array(b1, split=t))
            close(r, np.dot(a1, b1), rtol=1e-10)
    A, B = rng(3).standard_normal((7, 5)), rng(4).standard_normal((5, 9))
    for s in splits(2):
        for t in splits(2):
            close(ht.dot(ht.array(A, split=s), ht.array(B, split=t)), A @ B, rtol=1e-9, atol=1e-9)
    close(ht.dot(ht.array(A, split=0), 2.0), A * 2)
    out = ht.empty((7, 9), dtype=ht.float64)
    ht.dot(ht.array(A), ht.array(B), out=out)
    close(out, A @ B, rtol=1e-9, atol=1e-9)
    raises(NotImplementedError, ht.dot, ht.array(rng(5).standard_normal((2, 3, 4))), ht.array(a1[:4]))


def test_matmul():
    for (m, k, n) in ((7, 5, 9), (13, 8, 3), (2, 17, 5), (9, 1, 9)):
        A, B = rng(m).standard_normal((m, k)), rng(n).standard_normal((k, n))
        for s in splits(2):
            for t in splits(2):
                for dt, tol in ((np.float64, 1e-9), (np.float32, 1e-4)):
                    a, b = ht.array(A.astype(dt), split=s), ht.array(B.astype(dt), split=t)
                    r = ht.matmul(a, b)
                    assert r.gshape == (m, n)
                    close(r, A @ B, rtol=tol, atol=tol)
                    close(a @ b, A @ B, rtol=tol, atol=tol)
    # int x int stays int; mixed promotes
    Ai, Bi = rng(6).integers(-5, 5, (6, 4)), rng(7).integers(-5, 5, (4, 3))
    for s in splits(2):
        r = ht.matmul(ht.array(Ai, split=s), ht.array(Bi, split=s))
        same(r, Ai @ Bi)
        r = ht.matmul(ht.array(Ai.astype(np.int32), split=s), ht.array(Bi.astype(np.float32), split=s))
        assert r.dtype == ht.promote_types(ht.int32, ht.float32)
        close(r, Ai @ Bi)
    # vector operands
    A, v = rng(8).standard_normal((6, 4)), rng(9).standard_normal(4)
    for s in splits(2):
        for t in (None, 0):
            close(ht.matmul(ht.array(A, split=s), ht.array(v, split=t)), A @ v, rtol=1e-9)
            close(ht.matmul(ht.array(v, split=t), ht.array(A.T.copy(), split=s)), v @ A.T, rtol=1e-9)
    # batched
    X, Y = rng(10).standard_normal((3, 5, 4)), rng(11).standard_normal((3, 4, 6))
    for s in (None, 0):
        close(ht.matmul(ht.array(X, split=s), ht.array(Y, split=s)), X @ Y, rtol=1e-9, atol=1e-9)
    raises(ValueError, ht.matmul, ht.ones((25, 25)), ht.ones((42, 42)))


def test_matrix_norm():
    a = ht.arange(9, dtype=ht.float) - 4
    b = a.reshape((3, 3))
    B = b.numpy().astype(np.float64)
    for s in splits(2):
        bb = ht.array(B.astype(np.float32), split=s)
        for o in ("fro", 1, -1, np.inf, -np.inf):
            mn = ht.linalg.matrix_norm(bb, ord=o)
            assert mn.split is None and mn.dtype == ht.float32
            close(mn, np.linalg.norm(B, ord=o), rtol=1e-5)
        # ord 2 / -2 / nuc: the reference raises NotImplementedError; implemented here (SVD)
        for o in (2, -2, "nuc"):
            close(ht.linalg.matrix_norm(bb, ord=o), np.linalg.norm(B, ord=o), rtol=1e-4)
        mn = ht.linalg.matrix_norm(bb, keepdims=True)
        assert mn.shape == (1, 1)
    # tall and wide operands: the 2 / -2 / nuc norms come from the TSQR R factor when distributed
    for shape in ((41, 6), (6, 41)):
        T = rng(21).standard_normal(shape)
        for s in splits(2):
            for o in (2, -2, "nuc", "fro", 1, np.inf):
                close(ht.linalg.matrix_norm(ht.array(T, split=s), ord=o), np.linalg.norm(T, ord=o), rtol=1e-8)
    M = np.arange(18.0).reshape(2, 3, 3) - 9
    for s in splits(3):
        m = ht.array(M, split=s)
        mn = ht.linalg.matrix_norm(m, axis=(1, 2), ord=1)
        close(mn, np.linalg.norm(M, ord=1, axis=(1, 2)))
        mn = ht.linalg.matrix_norm(m, axis=(2, 1), ord=-np.inf)
        close(mn, np.linalg.norm(M, ord=-np.inf, axis=(2, 1)))
        if s == 0:
            assert mn.split == 0
    raises(ValueError, ht.linalg.matrix_norm, ht.ones((2, 2, 2)))
    raises(TypeError, ht.linalg.matrix_norm, ht.ones((2, 2)), axis=1)
    raises(TypeError, ht.linalg.matrix_norm, ht.ones((2, 2)), axis=(1, 2, 3))
    raises(ValueError, ht.linalg.matrix_norm, ht.array([1, 2, 3]))
    raises(ValueError, ht.linalg.matrix_norm, ht.ones((2, 2)), ord=3)


def test_vector_norm():
    v = rng(12).standard_normal(13)
    M = rng(13).standard_normal((5, 6))
    for s in (None, 0):
        x = ht.array(v, split=s)
        for o in (None, 1, 2, 3.5, np.inf, -np.inf, 0):
            r = ht.linalg.vector_norm(x, ord=o)
            close(r, np.linalg.norm(v, ord=2 if o is None else o), rtol=1e-9)
    for s in splits(2):
        x = ht.array(M, split=s)
        for ax in (0, 1, -1):
            for o in (1, 2, np.inf, -np.inf):
                r = ht.linalg.vector_norm(x, axis=ax, ord=o)
                close(r, np.linalg.norm(M, ord=o, axis=ax), rtol=1e-9)
                assert r.split == (None if s in (None, ax % 2) else (s if s < ax % 2 else s - 1))
        close(ht.linalg.vector_norm(x, keepdims=True), np.linalg.norm(M.reshape(-1)).reshape(1, 1), rtol=1e-9)
    c = ht.array([1 + 1j, 2 - 2j, 0 + 1j, 2 + 1j], dtype=ht.complex64, split=0)
    r = ht.linalg.vector_norm(c)
    assert r.dtype == ht.float32 and abs(float(r.item()) - 4.0) < 1e-6
    raises(ValueError, ht.vector_norm, ht.array([1, 2, 3]), ord="fro")
    raises(ValueError, ht.vector_norm, ht.array([1, 2, 3]), axis=(1, 2))
    raises(TypeError, ht.vector_norm, ht.array([1, 2, 3]), axis="r")


def test_norm():
    a = ht.arange(9, dtype=ht.float) - 4
    a0 = ht.array([1 + 1j, 2 - 2j, 0 + 1j, 2 + 1j], dtype=ht.complex64, split=0)
    gn = ht.linalg.norm(a, axis=0, ord=1)
    assert gn.split == a.split and gn.dtype == a.dtype and float(gn.item()) == 20.0
    gn = ht.linalg.norm(a0, keepdims=True)
    assert gn.split is None and gn.dtype == ht.float and abs(float(gn.item()) - 4.0) < 1e-6
    B = np.arange(9.0).reshape(3, 3) - 4
    for s in splits(2):
        b = ht.array(B.astype(np.float32), split=s)
        gn = ht.linalg.norm(b, ord="fro")
        assert gn.split is None
        close(gn, 7.745966692414834)
        close(ht.linalg.norm(b, ord=np.inf), 9.0)
        gn = ht.linalg.norm(b, axis=(0,), ord=-np.inf, keepdims=True)
        same(gn, np.array([[1.0, 0.0, 1.0]], dtype=np.float32))
        assert gn.split == s if s != 0 else gn.split is None
        close(ht.linalg.norm(b), np.linalg.norm(B))
    gn = ht.linalg.norm(ht.ones((3, 3, 3), dtype=ht.int), axis=(-2, -1))
    assert gn.split is None and gn.dtype == ht.float
    same(gn, np.array([3.0, 3.0, 3.0], dtype=np.float32))
    raises(ValueError, ht.linalg.norm, ht.ones(2), axis=(0, 1, 2))


def test_outer():
    a = ht.arange(3, dtype=ht.int32)
    b = ht.arange(8, dtype=ht.float32)
    npo = np.outer(np.arange(3), np.arange(8)).astype(np.float32)
    r = ht.outer(a, b, split=None)
    same(r, npo)
    assert r.larray.dtype == torch.einsum("i,j->ij", a.larray, b.larray).dtype
    a_s = ht.arange(3, dtype=ht.float32, split=0)
    b_s = ht.arange(8, dtype=ht.float32, split=0)
    r = ht.outer(a_s, b_s, split=1)
    assert r.split == 1
    same(r, npo)
    r = ht.outer(a_s, b_s, split=None)
    assert r.split == (0 if a_s.comm.size > 1 else r.split)
    same(r, npo)
    r = ht.outer(a, b_s, split=1)
    assert r.split == 1
    same(r, npo)
    r = ht.outer(a_s, b, split=0)
    assert r.split == 0
    same(r, npo)
    a3 = ht.array(rng(14).standard_normal((3, 3, 3)), split=2)
    r = ht.outer(a3, b_s)
    same(r, np.outer(a3.numpy(), np.arange(8.0, dtype=np.float32)))
    out = ht.empty((3, 8), dtype=ht.float32)
    ht.outer(a, b, out=out)
    same(out, npo)
    out = ht.empty((3, 8), dtype=ht.float32, split=1)
    ht.outer(a_s, b_s, out=out, split=1)
    same(out, npo)
    raises(TypeError, ht.outer, torch.arange(3), b)
    raises(TypeError, ht.outer, a, np.arange(8))
    raises(RuntimeError, ht.outer, ht.array(2.3), b)
    raises(TypeError, ht.outer, a, b, out=torch.empty((3, 8)))
    raises(ValueError, ht.outer, a, b, out=ht.empty((7, 8), dtype=ht.float32))
    raises(ValueError, ht.outer, a_s, b_s, out=ht.empty((3, 8), dtype=ht.float32, split=1), split=0)


def test_projection():
    a = ht.arange(1, 4, dtype=ht.float32, split=None)
    e1 = ht.array([1, 0, 0], dtype=ht.float32, split=None)
    assert ht.equal(ht.linalg.projection(a, e1), e1)
    a.resplit_(axis=0)
    assert ht.equal(ht.linalg.projection(a, e1), e1)
    e2 = ht.array([0, 1, 0], dtype=ht.float32, split=0)
    assert ht.equal(ht.linalg.projection(a, e2), e2 * 2)
    e3 = ht.array([0, 0, 1], dtype=ht.float32, split=0)
    assert ht.equal(ht.linalg.projection(ht.arange(1, 4, dtype=ht.float32), e3), e3 * 3)
    raises(TypeError, ht.linalg.projection, np.arange(1, 4), e1)
    raises(RuntimeError, ht.linalg.projection, ht.array([[1], [2], [3]], dtype=ht.float32), e1)


def test_trace():
    x_np = np.arange(24).reshape(6, 4)
    for s in splits(2):
        x = ht.array(x_np, split=s)
        r = ht.trace(x)
        assert isinstance(r, int) and r == np.trace(x_np)
        for o in (-7, -3, -1, 0, 1, 2, 4):
            assert ht.trace(x, offset=o) == np.trace(x_np, offset=o)
        r = ht.trace(x, dtype=ht.float32)
        assert isinstance(r, float) and r == float(np.trace(x_np))
        out = ht.empty((), dtype=ht.int64)
    x4 = np.arange(2 * 3 * 4 * 5).reshape(2, 3, 4, 5)
    for s in splits(4):
        x = ht.array(x4, split=s)
        for (a1, a2) in ((0, 1), (1, 3), (2, 0), (3, 2)):
            for o in (-1, 0, 2):
                r = ht.trace(x, offset=o, axis1=a1, axis2=a2)
                same(r, np.trace(x4, offset=o, axis1=a1, axis2=a2))
        out = ht.empty((4, 5), dtype=ht.int64)
        ht.trace(x, out=out)
        same(out, np.trace(x4))
    x = ht.arange(24).reshape((6, 4))
    raises(TypeError, ht.trace, "[[1, 2], [3, 4]]")
    raises(ValueError, ht.trace, ht.arange(24))
    raises(TypeError, ht.trace, x, axis1=0.2)
    raises(TypeError, ht.trace, x, axis2=1.4)
    raises(ValueError, ht.trace, x, axis1=2)
    raises(ValueError, ht.trace, x, axis2=2)
    raises(TypeError, ht.trace, x, offset=1.2)
    raises(ValueError, ht.trace, x, axis1=1, axis2=1)
    raises(ValueError, ht.trace, x, dtype="ht.int64")
    raises(TypeError, ht.trace, x, out=[])
    raises(ValueError, ht.trace, x, out=ht.array([]))


def test_transpose():
    x = rng(15).standard_normal((3, 4, 5))
    for s in splits(3):
        h = ht.array(x, split=s)
        for axes in (None, (0, 2, 1), (2, 0, 1), (1, 0, 2), (-1, 0, 1)):
            r = ht.transpose(h, axes) if axes is not None else h.T
            e = np.transpose(x, axes)
            same(r, e)
            if s is not None:
                perm = axes if axes is not None else (2, 1, 0)
                perm = [p % 3 for p in perm]
                assert r.split == perm.index(s)
    m = rng(16).standard_normal((5, 2))
    for s in splits(2):
        same(ht.array(m, split=s).transpose(), m.T)
    raises(TypeError, ht.transpose, 1)
    raises(TypeError, ht.transpose, ht.zeros((2, 3)), axes=1.0)
    raises(ValueError, ht.transpose, ht.zeros((2, 3)), axes=(-1,))
    raises(TypeError, ht.zeros((2, 3)).transpose, axes="01")
    raises(TypeError, ht.zeros((2, 3)).transpose, axes=(0, 1.0))
    raises((ValueError, IndexError), ht.zeros((2, 3)).transpose, axes=(0, 3))


def _tri(fn, npfn):
    for shape in ((7,), (6, 4), (4, 6), (5, 5), (2, 3, 4)):
        x = rng(17).standard_normal(shape)
        for s in splits(len(shape)):
            for k in (-2, -1, 0, 1, 3):
                r = fn(ht.array(x, split=s), k)
                if len(shape) == 1:
                    same(r, npfn(x, k))
                else:
                    same(r, npfn(x, k))
                    assert r.split == s
    raises(TypeError, fn, "asdf")
    raises(TypeError, fn, ht.ones((4, 4), split=0), ["sdf", "sf"])


def test_tril():
    _tri(ht.tril, np.tril)


def test_triu():
    _tri(ht.triu, np.triu)


def test_vecdot():
    a, b = rng(18).standard_normal((4, 5)), rng(19).standard_normal((4, 5))
    for s in splits(2):
        x, y = ht.array(a, split=s), ht.array(b, split=s)
        close(ht.vecdot(x, y), (a * b).sum(-1), rtol=1e-9)
        close(ht.vecdot(x, y, axis=0), (a * b).sum(0), rtol=1e-9)
        r = ht.vecdot(x, y, keepdim=True)
        assert r.gshape == (4, 1)
        close(r, (a * b).sum(-1, keepdims=True), rtol=1e-9)
    close(ht.vecdot(ht.array(a[0], split=0), ht.array(b[0], split=0)), np.dot(a[0], b[0]), rtol=1e-9)
