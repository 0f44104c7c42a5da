"""
Edge-case checks run at every world size of ``tests/test_distributed.py`` (1..8 ranks):

* empty ranks - arrays whose split extent is smaller than the world size (``p > gshape[split]``),
  so some ranks hold a (.., 0, ..) block. Reductions along other axes must keep the empty block,
  reductions along the split must not see phantom rows (ref ``_operations.py:401``);
* C-order of boolean-mask selection / ``nonzero`` on split > 0 arrays with data whose order
  would expose rank-block concatenation;
* owner-computes advanced indexing and ``__setitem__`` with distributed values (no gathers).

Every check compares against NumPy on the same global data.
"""
from __future__ import annotations

import numpy as np

import heat_amd as ht

from .dist_checks import assert_array_equal, for_splits


def _small_shapes():
    # split extents 1..3: at p >= 4 some ranks are empty for every split axis
    return [(3, 5), (5, 2), (2, 3, 4), (1, 6), (4, 1, 3)]


def check_empty_rank_reductions():
    rng = np.random.default_rng(11)
    for shp in _small_shapes():
        a = rng.standard_normal(shp)
        for s in for_splits(a):
            A = ht.array(a, split=s)
            assert_array_equal(ht.sum(A), a.sum())
            assert_array_equal(ht.max(A), a.max())
            assert_array_equal(ht.min(A), a.min())
            assert_array_equal(ht.prod(A), a.prod())
            for ax in range(a.ndim):
                assert_array_equal(ht.sum(A, axis=ax), a.sum(axis=ax))
                assert_array_equal(ht.max(A, axis=ax), a.max(axis=ax))
                assert_array_equal(ht.min(A, axis=ax), a.min(axis=ax))
                assert_array_equal(ht.prod(A, axis=ax), a.prod(axis=ax))
                assert_array_equal(ht.sum(A, axis=ax, keepdim=True), a.sum(axis=ax, keepdims=True))
                assert_array_equal(ht.argmax(A, axis=ax), a.argmax(axis=ax))
                assert_array_equal(ht.argmin(A, axis=ax), a.argmin(axis=ax))
                assert_array_equal(ht.cumsum(A, axis=ax), a.cumsum(axis=ax))
                assert_array_equal(ht.cumprod(A, axis=ax), a.cumprod(axis=ax))
                assert_array_equal(ht.all(A > -10, axis=ax), (a > -10).all(axis=ax))
                assert_array_equal(ht.any(A > 1, axis=ax), (a > 1).any(axis=ax))
            assert ht.argmax(A).item() == a.argmax()
            assert ht.argmin(A).item() == a.argmin()
            # chained: a reduction along a non-split axis followed by one along the split
            if a.ndim == 2:
                assert_array_equal(ht.sum(ht.max(A, axis=1)), a.max(axis=1).sum())
                assert_array_equal(ht.min(ht.sum(A, axis=0)), a.sum(axis=0).min())


def check_empty_rank_moments():
    rng = np.random.default_rng(12)
    for shp in _small_shapes():
        a = rng.standard_normal(shp)
        for s in for_splits(a):
            A = ht.array(a, split=s)
            assert_array_equal(ht.mean(A), a.mean())
            assert_array_equal(ht.var(A), a.var())
            assert_array_equal(ht.std(A, ddof=1), a.std(ddof=1) if a.size > 1 else np.nan)
            for ax in range(a.ndim):
                assert_array_equal(ht.mean(A, axis=ax), a.mean(axis=ax))
                assert_array_equal(ht.var(A, axis=ax), a.var(axis=ax))
                if a.shape[ax] > 1:
                    assert_array_equal(ht.std(A, axis=ax, ddof=1), a.std(axis=ax, ddof=1))
            if a.ndim == 2:
                assert_array_equal(ht.median(A, axis=0), np.median(a, axis=0))
                assert_array_equal(ht.median(A), np.median(a))
                assert_array_equal(ht.percentile(A, 30.0), np.percentile(a, 30.0), rtol=1e-6)


def check_empty_rank_manipulations():
    rng = np.random.default_rng(13)
    for shp in _small_shapes():
        a = rng.standard_normal(shp)
        ai = rng.integers(0, 3, size=shp)
        for s in for_splits(a):
            A = ht.array(a, split=s)
            for ax in range(a.ndim):
                v, _ = ht.sort(A, axis=ax)
                assert_array_equal(v, np.sort(a, axis=ax))
            u = ht.unique(ht.array(ai, split=s), sorted=True)
            assert_array_equal(u, np.unique(ai))
            assert_array_equal(ht.resplit(A, None), a)
            for t in range(a.ndim):
                assert_array_equal(ht.resplit(A, t), a)
            assert_array_equal(ht.flip(A, 0), np.flip(a, 0))
            assert_array_equal(ht.roll(A, 1, axis=0), np.roll(a, 1, axis=0))
            assert_array_equal(ht.reshape(A, (-1,), new_split=0), a.reshape(-1))
            assert_array_equal(ht.concatenate([A, A], axis=0), np.concatenate([a, a], axis=0))
            assert_array_equal(A.T if a.ndim == 2 else ht.transpose(A), a.T)
            B = A.copy()
            B.balance_()
            assert_array_equal(B, a)


def check_empty_rank_indexing():
    rng = np.random.default_rng(14)
    for shp in _small_shapes():
        a = rng.standard_normal(shp)
        for s in for_splits(a):
            A = ht.array(a, split=s)
            assert_array_equal(A[0], a[0])
            assert_array_equal(A[-1], a[-1])
            assert_array_equal(A[1:], a[1:], check_split_chunks=False)
            assert_array_equal(A[A > 0], a[a > 0], check_split_chunks=False)
            assert_array_equal(ht.nonzero(A > 0), np.argwhere(a > 0), check_split_chunks=False)
            B = ht.array(a, split=s)
            B[B > 0] = 0.0
            b = a.copy()
            b[b > 0] = 0.0
            assert_array_equal(B, b)
            B[0] = 7.0
            b[0] = 7.0
            assert_array_equal(B, b)
            B[..., -1] = -3.0
            b[..., -1] = -3.0
            assert_array_equal(B, b)


def check_empty_rank_linalg():
    rng = np.random.default_rng(15)
    for m, k, n in [(3, 2, 5), (2, 6, 3), (1, 3, 1), (5, 1, 2)]:
        a = rng.standard_normal((m, k))
        b = rng.standard_normal((k, n))
        for sa in (None, 0, 1):
            for sb in (None, 0, 1):
                C = ht.matmul(ht.array(a, split=sa), ht.array(b, split=sb))
                assert_array_equal(C, a @ b, rtol=1e-5, atol=1e-8, check_split_chunks=False)
        for s in (None, 0, 1):
            A = ht.array(a, split=s)
            for ordv in (None, "fro", 1, -1, np.inf, -np.inf):
                got = ht.linalg.matrix_norm(A, ord=ordv) if ordv is not None else ht.linalg.norm(A)
                exp = np.linalg.norm(a, ord=ordv)
                assert abs(float(got.item()) - exp) < 1e-8 * max(1.0, abs(exp)), (ordv, s, got, exp)
            v = rng.standard_normal(k)
            assert_array_equal(ht.matmul(A, ht.array(v, split=0)), a @ v, check_split_chunks=False)
            assert abs(float(ht.linalg.trace(A)) - np.trace(a)) < 1e-10
            x = rng.standard_normal(m)
            X = ht.array(x, split=0)
            assert abs(ht.dot(X, X).item() - x @ x) < 1e-10
            assert abs(ht.linalg.vector_norm(X).item() - np.linalg.norm(x)) < 1e-10


# ---------------------------------------------------------------------------------------------
def check_mask_order_split_gt0():
    """Data whose values equal their C-order position: any rank-order concatenation shows."""
    for shp in [(3, 4), (2, 5, 3), (6, 7), (1, 9)]:
        a = np.arange(int(np.prod(shp))).reshape(shp)
        for s in for_splits(a):
            A = ht.array(a, split=s)
            for t in (2, 5, 11):
                assert_array_equal(A[A > t], a[a > t], check_split_chunks=False)
                assert_array_equal(A[(A % 3) == 0], a[(a % 3) == 0], check_split_chunks=False)
                assert_array_equal(ht.nonzero(A > t), np.argwhere(a > t), check_split_chunks=False)
            # masked assignment with an array value in C order of the True positions
            B = ht.array(a, split=s)
            msk = a % 2 == 1
            vals = -np.arange(int(msk.sum()))
            B[B % 2 == 1] = ht.array(vals, split=0)
            b = a.copy()
            b[msk] = vals
            assert_array_equal(B, b)
            B = ht.array(a, split=s)
            B[B % 2 == 1] = ht.array(vals)  # replicated value
            assert_array_equal(B, b)


def check_advanced_indexing_owner_computes():
    rng = np.random.default_rng(16)
    a = rng.standard_normal((7, 6, 5))
    idx0 = np.array([6, 0, 3, 3, 1])
    idx1 = np.array([5, 2, 0, 1, 4])
    for s in for_splits(a):
        A = ht.array(a, split=s)
        assert_array_equal(A[idx0, idx1], a[idx0, idx1], check_split_chunks=False)
        assert_array_equal(A[idx0, :, idx1[:5] % 5], a[idx0, :, idx1[:5] % 5], check_split_chunks=False)
        assert_array_equal(A[:, idx1, 2], a[:, idx1, 2], check_split_chunks=False)
        assert_array_equal(A[idx0[:, None], idx1[None, :3]], a[idx0[:, None], idx1[None, :3]],
                           check_split_chunks=False)
        m2 = a[:, :, 0] > 0
        assert_array_equal(A[m2], a[m2], check_split_chunks=False)
        assert_array_equal(A[2, idx1], a[2, idx1], check_split_chunks=False)


def check_setitem_distributed_value():
    rng = np.random.default_rng(17)
    a = rng.standard_normal((9, 6))
    for s in for_splits(a):
        for vs in (None, 0, 1):
            # slice along the split axis with a distributed value of the selection's shape
            A = ht.array(a, split=s)
            v = rng.standard_normal((5, 6))
            A[2:7] = ht.array(v, split=vs)
            b = a.copy()
            b[2:7] = v
            assert_array_equal(A, b)
            A = ht.array(a, split=s)
            w = rng.standard_normal((9, 3))
            A[:, 1:4] = ht.array(w, split=vs)
            b = a.copy()
            b[:, 1:4] = w
            assert_array_equal(A, b)
            A = ht.array(a, split=s)
            A[::2, ::3] = ht.array(rng.standard_normal((5, 2)), split=vs) * 0 + 1.5
            b = a.copy()
            b[::2, ::3] = 1.5
            assert_array_equal(A, b)
            # integer index arrays
            A = ht.array(a, split=s)
            idx = np.array([8, 1, 4])
            u = rng.standard_normal((3, 6))
            A[idx] = ht.array(u, split=vs)
            b = a.copy()
            b[idx] = u
            assert_array_equal(A, b)
            A = ht.array(a, split=s)
            A[idx, np.array([0, 5, 2])] = ht.array(np.array([1.0, 2.0, 3.0]), split=None if vs == 1 else vs)
            b = a.copy()
            b[idx, np.array([0, 5, 2])] = [1.0, 2.0, 3.0]
            assert_array_equal(A, b)
        # broadcast value (local), the general path
        A = ht.array(a, split=s)
        A[np.array([0, 3]), np.array([1, 2])] = 9.0
        b = a.copy()
        b[np.array([0, 3]), np.array([1, 2])] = 9.0
        assert_array_equal(A, b)


def check_different_split_binary_ops():
    """Intentional extension: operands split along different axes are aligned with one
    all-to-all (the reference raises NotImplementedError, ``_operations.py:104-107``)."""
    rng = np.random.default_rng(18)
    a = rng.standard_normal((6, 5, 4))
    b = rng.standard_normal((6, 5, 4))
    for sa in range(3):
        for sb in range(3):
            C = ht.array(a, split=sa) * ht.array(b, split=sb)
            assert C.split == sa
            assert_array_equal(C, a * b)
    # broadcast operand of lower rank with a different split
    c = rng.standard_normal((5, 4))
    assert_array_equal(ht.array(a, split=0) + ht.array(c, split=1), a + c)


def check_lasso_mismatched_y_layouts():
    """y distributed differently from x (split None vs 0, (m,1) split 1, unbalanced
    split 0) must give the same fit, never an out-of-bounds read of y in the native kernels."""
    import os

    rng = np.random.default_rng(19)
    m, n = 97, 5
    X = rng.normal(size=(m, n)).astype(np.float32)
    X /= np.sqrt((X ** 2).mean(0))
    w = np.array([0.5, 2.0, 0.0, -1.5, 0.7], np.float32)
    y = (X @ w + 0.01 * rng.normal(size=m)).astype(np.float32)
    prev = os.environ.get("HEAT_LASSO_SOLVER")
    ref = None
    try:
        for solver in ("sweep", "gram"):
            os.environ["HEAT_LASSO_SOLVER"] = solver
            for xs, ys, yshape in ((0, None, (m, 1)), (None, 0, (m,)), (0, 1, (1, m)), (0, 1, (m, 1)),
                                   (None, 1, (1, m)), (0, "unbal", (m,))):
                yv = y.reshape(yshape)
                if ys == "unbal":
                    Y = ht.array(yv, split=0)[3:]
                    Y = ht.concatenate([ht.array(yv[:3]), Y])  # unbalanced distribution of the same y
                else:
                    Y = ht.array(yv, split=ys if not (ys == 1 and yshape[1] == 1) else 1)
                est = ht.regression.Lasso(lam=0.01, max_iter=100, tol=1e-8)
                est.fit(ht.array(X, split=xs), Y)
                th = est.theta.numpy().ravel()
                if ref is None:
                    ref = th
                assert np.allclose(th, ref, atol=1e-4), (solver, xs, ys, yshape, th, ref)
        bad = ht.array(y[:-1], split=0)
        try:
            ht.regression.Lasso(max_iter=2).fit(ht.array(X, split=0), bad)
            raise AssertionError("a y of the wrong length must raise")
        except ValueError:
            pass
    finally:
        if prev is None:
            os.environ.pop("HEAT_LASSO_SOLVER", None)
        else:
            os.environ["HEAT_LASSO_SOLVER"] = prev


def check_nonblocking_v_collectives():
    """Ialltoallv / Igatherv / Iscatterv return a pending request: several can be in flight at once
    and complete in any Wait order (round 1 completed them synchronously)."""
    import torch

    comm = ht.MPI_WORLD
    p, r = comm.size, comm.rank
    # all-to-all of rank-dependent blocks, two requests in flight
    send1 = torch.arange(p * 3, dtype=torch.float64).reshape(p * 3, 1) + 100 * r
    recv1 = torch.empty(p * 3, 1, dtype=torch.float64)
    send2 = torch.full((p * 2, 4), float(r), dtype=torch.float32)
    recv2 = torch.empty(p * 2, 4, dtype=torch.float32)
    q1 = comm.Ialltoallv(send1, recv1)
    q2 = comm.Ialltoallv(send2, recv2)
    q2.Wait()
    q1.Wait()
    for src in range(p):
        assert torch.equal(recv1[3 * src: 3 * src + 3, 0], torch.arange(3 * r, 3 * r + 3, dtype=torch.float64) + 100 * src)
        assert torch.all(recv2[2 * src: 2 * src + 2] == src)
    # gather of unequal blocks to root 0 and a scatter back, overlapped
    blk = torch.full((r + 1, 2), float(r))
    tot = sum(range(1, p + 1))
    g = torch.empty(tot, 2) if r == 0 else None
    qg = comm.Igatherv(blk, g, root=0)
    sc_recv = torch.empty(2, 3)
    sc_send = torch.arange(p * 6, dtype=torch.float32).reshape(p * 2, 3) if r == 0 else None
    qs = comm.Iscatterv(sc_send, sc_recv, root=0)
    qs.Wait()
    qg.Wait()
    assert torch.equal(sc_recv, torch.arange(6 * r, 6 * r + 6, dtype=torch.float32).reshape(2, 3))
    if r == 0:
        exp = torch.cat([torch.full((q + 1, 2), float(q)) for q in range(p)])
        assert torch.equal(g, exp)


def check_qr_ill_conditioned_householder():
    """cond(A) = 1e12 (fp64): CholeskyQR2 breaks down, the distributed Householder path must give
    an orthogonal Q and A = QR on every split."""
    rng = np.random.default_rng(20)
    for m, n in ((120, 17), (64, 40), (300, 33)):
        u, _ = np.linalg.qr(rng.standard_normal((m, n)))
        v, _ = np.linalg.qr(rng.standard_normal((n, n)))
        a = (u * np.logspace(0, -12, n)) @ v.T
        for s in (None, 0):
            q, r = ht.linalg.qr(ht.array(a, split=s), mode="reduced")
            qn, rn = q.numpy(), r.numpy()
            assert np.abs(qn.T @ qn - np.eye(n)).max() < 1e-12, np.abs(qn.T @ qn - np.eye(n)).max()
            assert np.abs(qn @ rn - a).max() < 1e-12 * np.abs(a).max() * 10
            assert np.allclose(rn, np.triu(rn))


def check_netcdf_modes_unlimited_slices():
    """save_netcdf without netCDF4 (classic CDF-2): mode 'w' / 'a' / 'r+', several variables per
    file, an unlimited (record) dimension grown by later writes, and file_slices - parity with the
    reference's netCDF4 path (io.py:348-650), every rank writing its slab in place."""
    import os
    import tempfile

    comm = ht.MPI_WORLD
    d = comm.bcast(tempfile.mkdtemp(prefix="ht_nc_") if comm.rank == 0 else None, root=0)
    a = np.arange(7 * 5, dtype=np.float32).reshape(7, 5)
    p = os.path.join(d, "m.nc")
    for s in (None, 0, 1):
        ht.save_netcdf(ht.array(a, split=s), p, "x", mode="w")
        assert np.array_equal(ht.load_netcdf(p, "x").numpy(), a)
        ht.save_netcdf(ht.array(2 * a, split=s), p, "y", mode="a", dimension_names=["r", "c"])
        assert np.array_equal(ht.load_netcdf(p, "y", split=0).numpy(), 2 * a)
        assert np.array_equal(ht.load_netcdf(p, "x").numpy(), a)        # untouched by the append
        ht.save_netcdf(ht.array(a[:3] + 100, split=s), p, "x", mode="r+", file_slices=slice(2, 5))
        exp = a.copy()
        exp[2:5] = a[:3] + 100
        assert np.array_equal(ht.load_netcdf(p, "x").numpy(), exp)
        ht.save_netcdf(ht.array(a[:, 1] - 1, split=0 if s is not None else None), p, "x", mode="r+",
                       file_slices=(slice(None), 1))
        exp[:, 1] = a[:, 1] - 1
        assert np.array_equal(ht.load_netcdf(p, "x").numpy(), exp)
    q = os.path.join(d, "u.nc")
    ht.save_netcdf(ht.array(a, split=0), q, "z", is_unlimited=True, dimension_names=["t", "c"])
    ht.save_netcdf(ht.array(a[:4] + 50, split=0), q, "z", mode="a", file_slices=slice(7, 11))
    z = ht.load_netcdf(q, "z").numpy()
    assert z.shape == (11, 5) and np.array_equal(z[:7], a) and np.array_equal(z[7:], a[:4] + 50)
    comm.Barrier()
    for bad in (lambda: ht.save_netcdf(ht.array(a), p, "x", mode="x"),
                lambda: ht.save_netcdf(ht.array(a), p, "x", dimension_names=["only_one"])):
        try:
            bad()
            raise AssertionError("must raise")
        except ValueError:
            pass


def check_matmul_ring_streamed():
    """Panel-streamed matmul (``linalg/basics.py`` ring path, threshold forced to 0) for every
    split pair, including ranks that hold empty panels (p > the split extent)."""
    from heat_amd.core.linalg import basics

    old = basics._RING_MIN_BYTES
    basics._RING_MIN_BYTES = 0
    try:
        rng = np.random.default_rng(61)
        for (m, k, n) in ((9, 7, 5), (3, 2, 4), (17, 1, 6)):
            a = rng.standard_normal((m, k))
            b = rng.standard_normal((k, n))
            for sa in (None, 0, 1):
                for sb in (None, 0, 1):
                    C = ht.array(a, split=sa) @ ht.array(b, split=sb)
                    assert np.allclose(C.numpy(), a @ b, rtol=1e-10, atol=1e-12), (m, k, n, sa, sb)
                    if sa == 0 and sb in (0, 1):
                        assert C.split == 0
            v = rng.standard_normal(k)
            V = ht.array(v, split=0)
            assert np.allclose(ht.matmul(ht.array(a, split=1), V).numpy(), a @ v)
            assert np.allclose(ht.matmul(ht.array(a, split=0), V).numpy(), a @ v)
    finally:
        basics._RING_MIN_BYTES = old


def check_matmul_ring_direct():
    """The all-peers ring mode (``HEAT_RING_MODE=direct``: every block posted to all p - 1 peers
    at once) gives the same panel-streamed matmul and streamed cdist as the neighbour ring."""
    import os

    from heat_amd.core.linalg import basics

    old, old_env = basics._RING_MIN_BYTES, os.environ.get("HEAT_RING_MODE")
    basics._RING_MIN_BYTES = 0
    os.environ["HEAT_RING_MODE"] = "direct"
    try:
        rng = np.random.default_rng(62)
        for (m, k, n) in ((9, 7, 5), (17, 1, 6), (3, 4, 2)):
            a = rng.standard_normal((m, k))
            b = rng.standard_normal((k, n))
            for sa in (0, 1):
                for sb in (0, 1):
                    C = ht.array(a, split=sa) @ ht.array(b, split=sb)
                    assert np.allclose(C.numpy(), a @ b, rtol=1e-10, atol=1e-12), (m, k, n, sa, sb)
        x = rng.standard_normal((23, 3)).astype(np.float32)
        X = ht.array(x, split=0)
        seen = []
        ht.spatial.cdist_stream(X, X, lambda d, i, j: seen.append((i, j, d.shape)), tile=5)
        rows = sum(s[0] for (i, j, s) in seen if j == 0)
        assert rows == X.lshape[0]
        d = ht.spatial.cdist(X, X)
        ref = np.sqrt(((x[:, None, :] - x[None, :, :]) ** 2).sum(-1))
        assert np.allclose(d.numpy(), ref, atol=1e-4)
    finally:
        basics._RING_MIN_BYTES = old
        if old_env is None:
            os.environ.pop("HEAT_RING_MODE", None)
        else:
            os.environ["HEAT_RING_MODE"] = old_env


def check_qr_split1_panels():
    """Column-split QR keeps the column split (Householder panel factorisation by the owner,
    reflector broadcasts): orthogonal Q, A = QR, upper-triangular R, also for cond(A) = 1e10 and
    for ranks with no columns."""
    rng = np.random.default_rng(23)
    for m, n, cond in ((120, 17, 1.0), (64, 40, 1e10), (50, 50, 1e3), (40, 3, 1.0)):
        u, _ = np.linalg.qr(rng.standard_normal((m, n)))
        v, _ = np.linalg.qr(rng.standard_normal((n, n)))
        a = (u * np.logspace(0, -np.log10(cond), n)) @ v.T
        for mode in ("reduced", None):
            if mode is None and m != n:
                continue
            q, r = ht.linalg.qr(ht.array(a, split=1), mode=mode or "complete")
            assert q.split == 1 and r.split == 1
            qn, rn = q.numpy(), r.numpy()
            assert np.abs(qn.T @ qn - np.eye(n)).max() < 1e-12, np.abs(qn.T @ qn - np.eye(n)).max()
            assert np.abs(qn @ rn - a).max() < 1e-12 * np.abs(a).max() * 10
            assert np.allclose(rn, np.triu(rn))
            assert np.all(np.diag(rn) >= 0)
            _, r_only = ht.linalg.qr(ht.array(a, split=1), mode="reduced", calc_q=False)
            assert np.allclose(r_only.numpy(), rn, atol=1e-10)


def check_svd_layouts():
    """svd: tall split 0 (TSQR + SVD of R), wide split 1 (the same on the transpose), gathered
    otherwise; singular values vs NumPy, U S V^T reconstructs A, U and V orthonormal."""
    rng = np.random.default_rng(5)
    for shp, split in [((40, 6), 0), ((6, 40), 1), ((40, 6), None), ((12, 9), 1), ((9, 12), 0)]:
        a_np = rng.standard_normal(shp)
        a = ht.array(a_np, split=split)
        s_only = ht.linalg.svd(a, compute_uv=False)
        np.testing.assert_allclose(s_only.numpy(), np.linalg.svd(a_np, compute_uv=False), rtol=1e-10, atol=1e-10)
        u, s, v = ht.linalg.svd(a)
        un, sn, vn = u.numpy(), s.numpy(), v.numpy()
        r = min(shp)
        assert un.shape == (shp[0], r) and vn.shape == (shp[1], r) and sn.shape == (r,)
        np.testing.assert_allclose(sn, np.linalg.svd(a_np, compute_uv=False), rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose((un * sn) @ vn.T, a_np, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(un.T @ un, np.eye(r), atol=1e-9)
        np.testing.assert_allclose(vn.T @ vn, np.eye(r), atol=1e-9)
    raises_ok = False
    try:
        ht.linalg.svd(ht.zeros((2, 3, 4)))
    except ValueError:
        raises_ok = True
    assert raises_ok


def check_diag_unique_without_gather():
    """``diag`` of a split vector (one redistribution of the vector into the result's row blocks)
    and ``unique(axis=...)`` (local uniques + one all-gather of them, inverse from the global
    uniques) on every split, against numpy."""
    rng = np.random.default_rng(4)
    for m in (1, 5, 11):
        v = rng.standard_normal(m)
        for off in (-3, -1, 0, 2, 4):
            for s in (None, 0):
                d = ht.diag(ht.array(v, split=s), off)
                assert np.allclose(d.numpy(), np.diag(v, off)), (m, off, s)
                if s == 0:
                    assert d.split == 0
    a = rng.integers(0, 3, (23, 4)).astype(np.float32)
    for s in (None, 0, 1):
        for ax in (0, 1):
            x = ht.array(a, split=s)
            u, inv = ht.unique(x, return_inverse=True, axis=ax)
            ru, rinv = np.unique(a, axis=ax, return_inverse=True)
            assert np.allclose(u.numpy(), ru), (s, ax)
            assert np.array_equal(inv.numpy().reshape(-1), rinv.reshape(-1)), (s, ax)


def check_knn_custom_metric_candidates():
    """kNN with a user metric whose distance matrix is column-split (replicated queries vs split
    training rows): per-rank top-k candidates + one all-gather, no gather of the matrix; labels
    equal a numpy brute force."""
    rng = np.random.default_rng(8)
    xt = rng.standard_normal((41, 3)).astype(np.float32)
    yt = rng.integers(0, 3, 41)
    onehot = np.eye(3, dtype=np.float32)[yt]
    q = rng.standard_normal((9, 3)).astype(np.float32)
    knn = ht.classification.KNeighborsClassifier(n_neighbors=4,
                                                 effective_metric_=lambda a, b: ht.spatial.cdist(a, b))
    knn.fit(ht.array(xt, split=0), ht.array(onehot, split=0))
    pred = knn.predict(ht.array(q)).numpy()
    d = np.sqrt(((q[:, None, :] - xt[None]) ** 2).sum(-1))
    nn = np.argsort(d, axis=1, kind="stable")[:, :4]
    ref = np.argmax(onehot[nn].sum(1), axis=1)
    assert np.array_equal(pred, ref), (pred, ref)


def check_qr_complete_without_gather():
    """Complete-mode QR (Q m x m) of tall, square and wide matrices on every split: orthogonal
    Q, Q R = A, R upper trapezoidal with a non-negative diagonal, Q split 0 (1 for split-1
    input) - formed by the distributed Householder path, no gather of A or Q."""
    rng = np.random.default_rng(17)
    for (m, n) in ((13, 4), (9, 9), (5, 11), (3, 3), (20, 1)):
        a = rng.standard_normal((m, n))
        for s in (0, 1):
            q, r = ht.linalg.qr(ht.array(a, split=s), mode="complete")
            Q, R = q.numpy(), r.numpy()
            assert Q.shape == (m, m) and R.shape == (m, n), (m, n, s)
            assert np.allclose(Q.T @ Q, np.eye(m), atol=1e-5), (m, n, s)
            assert np.allclose(Q @ R, a, atol=1e-5), (m, n, s)
            assert np.allclose(np.tril(R, -1), 0, atol=1e-6)
            k = min(m, n)
            assert (np.diagonal(R)[:k] >= -1e-7).all()
            assert q.split == (0 if s == 0 else 1) and r.split == s


def check_kmeans_bit_reproducible():
    """Two fits with the same seed give bit-identical centroids, labels and inertia on every rank
    (the deterministic update: no float atomics, fixed-order partial sums), the centroids are the
    same on all ranks, and the labels are the nearest centroids (NumPy fp64 check, ties aside).
    k = 40 takes the MFMA assignment + counting-sort update on a GPU, k = 8 the fused small-k step."""
    import torch

    rng = np.random.default_rng(21)
    centres = rng.standard_normal((40, 16)) * 6
    pts = (centres[rng.integers(0, 40, 6000)] + rng.standard_normal((6000, 16))).astype(np.float32)
    for k in (40, 8):
        runs = []
        for _ in range(2):
            X = ht.array(pts, split=0)
            km = ht.cluster.KMeans(n_clusters=k, init="random", max_iter=12, tol=None, random_state=5)
            km.fit(X)
            runs.append((km.cluster_centers_.larray.clone(), km.labels_.larray.clone(), float(km.inertia_)))
        (c0, l0, i0), (c1, l1, i1) = runs
        assert torch.equal(c0, c1), (k, (c0 - c1).abs().max())
        assert torch.equal(l0, l1) and i0 == i1
        # replicated centroids: identical bits on every rank
        gathered = X.comm.allgather_tensor(c0.reshape(1, -1).contiguous(), 0)
        assert all(torch.equal(gathered[0], g) for g in gathered)
        # labels_ belong to the last assignment (against the centroids before the final update,
        # as in the reference); predict() assigns against the final ones
        lab = km.predict(X).numpy().reshape(-1)
        c = km.cluster_centers_.numpy().astype(np.float64)
        d = ((pts.astype(np.float64)[:, None, :] - c[None]) ** 2).sum(-1)
        best = d.min(1)
        assert np.all(d[np.arange(len(pts)), lab] <= best * (1 + 1e-5) + 1e-4)


def check_cdist_symmetric_half_ring():
    """cdist(X) / rbf(X) / manhattan(X) with X split 0 and no Y through the half ring (every
    off-diagonal tile computed once, its transpose sent back; reference spatial/distance.py:265-362)
    equal the NumPy distance matrix, for uneven blocks and every p (odd and even last step)."""
    import os

    from scipy.spatial.distance import cdist as sp_cdist

    comm = ht.MPI_WORLD
    rng = np.random.default_rng(5)
    old = os.environ.get("HEAT_CDIST_ALLGATHER_BYTES")
    os.environ["HEAT_CDIST_ALLGATHER_BYTES"] = "0"      # force the ring paths
    try:
        for n in (3 * comm.size + 2, 2 * comm.size - 1):
            a = rng.standard_normal((n, 5)).astype(np.float64)
            X = ht.array(a, split=0)
            ref = sp_cdist(a, a)
            d = ht.spatial.cdist(X)
            assert d.split == 0 and d.shape == (n, n)
            np.testing.assert_allclose(d.numpy(), ref, atol=1e-9)
            np.testing.assert_allclose(ht.spatial.cdist(X, X).numpy(), ref, atol=1e-9)   # full ring
            np.testing.assert_allclose(ht.spatial.rbf(X, sigma=1.5).numpy(), np.exp(-ref ** 2 / (2 * 1.5 ** 2)),
                                       atol=1e-9)
            np.testing.assert_allclose(ht.spatial.manhattan(X).numpy(), sp_cdist(a, a, "cityblock"), atol=1e-9)
            d32 = ht.spatial.cdist(ht.array(a.astype(np.float32), split=0), quadratic_expansion=True)
            np.testing.assert_allclose(d32.numpy(), ref, atol=2e-3)
    finally:
        if old is None:
            os.environ.pop("HEAT_CDIST_ALLGATHER_BYTES", None)
        else:
            os.environ["HEAT_CDIST_ALLGATHER_BYTES"] = old
