"""
Randomised differential checks: seeded random cases (the same on every rank), each a random shape,
dtype and split axis, against NumPy. Where ``dist_checks`` pins every operation on hand-picked
data, these sweep the layout space - uneven blocks, split extents smaller than the world (empty
ranks), length-1 axes, negative axes, keepdims - the way the reference's ``assert_func_equal``
draws random arrays for every split (``heat/core/tests/test_suites/basic_test.py:142-306``).

Run in a world of one (``test_core_local.py``), at 2-8 gloo ranks and host-staged
(``test_distributed.py``), and with device buffers on the GPU (``test_gpu_dist.py``).
"""
from __future__ import annotations

import numpy as np

import heat_amd as ht

from .dist_checks import assert_array_equal

N_CASES = 12


def _cases(seed, n=N_CASES, max_ndim=3, max_extent=7, float_only=False):
    """(numpy array, split) pairs: random ndim 1..max_ndim, extents 1..max_extent, dtype, split."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        nd = int(rng.integers(1, max_ndim + 1))
        shape = tuple(int(v) for v in rng.integers(1, max_extent + 1, nd))
        kind = "f" if float_only else rng.choice(["f", "d", "i"])
        if kind == "i":
            a = rng.integers(-20, 20, shape).astype(np.int64)
        else:
            a = rng.standard_normal(shape).astype(np.float32 if kind == "f" else np.float64)
        split = None if rng.random() < 0.2 else int(rng.integers(0, nd))
        out.append((a, split))
    return out, rng


def _tol(a):
    return (1e-4, 1e-5) if a.dtype == np.float32 else (1e-9, 1e-10)


def check_random_elementwise():
    cases, rng = _cases(101)
    for a, split in cases:
        x = ht.array(a, split=split)
        rt, at = _tol(a)
        b = rng.standard_normal(a.shape[-1:]).astype(a.dtype) if a.dtype.kind == "f" else \
            rng.integers(1, 5, a.shape[-1:]).astype(a.dtype)
        y = ht.array(b)  # replicated, broadcast along the last axis
        assert_array_equal(x + y, a + b, rtol=rt, atol=at)
        assert_array_equal(x * y - x, a * b - a, rtol=rt, atol=at)
        assert_array_equal(ht.abs(x), np.abs(a), rtol=rt, atol=at)
        assert_array_equal(x > 0, a > 0)
        assert_array_equal(ht.where(x > 0, x, 0), np.where(a > 0, a, 0), rtol=rt, atol=at)
        if a.dtype.kind == "f":
            assert_array_equal(ht.exp(ht.clip(x, -3, 3)), np.exp(np.clip(a, -3, 3)), rtol=rt, atol=at)
            assert_array_equal(ht.sqrt(ht.abs(x)), np.sqrt(np.abs(a)), rtol=rt, atol=at)
        else:
            assert_array_equal(x // 3, a // 3)
            assert_array_equal(x % 4, a % 4)


def check_random_reductions():
    cases, rng = _cases(202)
    for a, split in cases:
        x = ht.array(a, split=split)
        rt, at = _tol(a)
        rt, at = rt * 10, at * 10
        ax = int(rng.integers(-a.ndim, a.ndim))
        keep = bool(rng.random() < 0.5)
        assert_array_equal(ht.sum(x, axis=ax, keepdim=keep), a.sum(axis=ax, keepdims=keep), rtol=rt, atol=at,
                           check_split_chunks=False)
        assert_array_equal(ht.max(x, axis=ax, keepdim=keep), a.max(axis=ax, keepdims=keep), check_split_chunks=False)
        assert_array_equal(ht.min(x, axis=ax), a.min(axis=ax), check_split_chunks=False)
        assert_array_equal(ht.argmax(x, axis=ax), a.argmax(axis=ax), check_split_chunks=False)
        assert_array_equal(ht.argmin(x, axis=ax), a.argmin(axis=ax), check_split_chunks=False)
        if a.dtype.kind == "f":
            assert_array_equal(ht.mean(x, axis=ax), a.mean(axis=ax), rtol=rt, atol=at, check_split_chunks=False)
            if a.shape[ax] > 1:
                assert_array_equal(ht.var(x, axis=ax, ddof=1), a.var(axis=ax, ddof=1), rtol=rt * 10, atol=at * 10,
                                   check_split_chunks=False)
            assert abs(float(ht.mean(x)) - float(a.mean())) <= 1e-4 * (1 + abs(float(a.mean())))
        assert abs(float(ht.sum(x)) - float(a.sum())) <= 1e-3 * (1 + float(np.abs(a).sum()))


def check_random_manipulations():
    cases, rng = _cases(303)
    for a, split in cases:
        x = ht.array(a, split=split)
        perm = tuple(int(v) for v in rng.permutation(a.ndim))
        assert_array_equal(ht.transpose(x, perm), np.transpose(a, perm), check_split_chunks=False)
        ax = int(rng.integers(0, a.ndim))
        assert_array_equal(ht.flip(x, ax), np.flip(a, ax), check_split_chunks=False)
        sh = int(rng.integers(-5, 6))
        assert_array_equal(ht.roll(x, sh, ax), np.roll(a, sh, ax), check_split_chunks=False)
        assert_array_equal(ht.concatenate([x, x], axis=ax), np.concatenate([a, a], axis=ax), check_split_chunks=False)
        # the split must name an axis of the new shape (reference reshape: new_split defaults to
        # the old split and is sanitised against the new shape)
        ns = None if split is None else 0
        flat = ht.reshape(x, (-1,), new_split=ns)
        assert_array_equal(flat, a.reshape(-1), check_split_chunks=False)
        n = a.size
        div = [d for d in range(1, n + 1) if n % d == 0]
        d = int(rng.choice(div))
        ns = None if split is None else int(rng.integers(0, 2))
        r2 = ht.reshape(x, (d, n // d), new_split=ns)
        assert r2.split == ns
        assert_array_equal(r2, a.reshape(d, n // d))
        srt = ht.sort(x, axis=ax)[0]
        assert_array_equal(srt, np.sort(a, axis=ax, kind="stable"), check_split_chunks=False)
        assert_array_equal(ht.expand_dims(x, 0), a[None], check_split_chunks=False)
        if split is not None:
            new = int(rng.integers(0, a.ndim))
            r = ht.resplit(x, new)
            assert r.split == new
            assert_array_equal(r, a)


def check_random_indexing():
    cases, rng = _cases(404)
    for a, split in cases:
        x = ht.array(a, split=split)
        key = []
        for s in a.shape:
            lo = int(rng.integers(0, s))
            hi = int(rng.integers(lo, s + 1))
            step = int(rng.integers(1, 3))
            key.append(slice(lo, hi, step))
        key = tuple(key)
        assert_array_equal(x[key], a[key], check_split_chunks=False)
        i = int(rng.integers(-a.shape[0], a.shape[0]))
        assert_array_equal(x[i], a[i], check_split_chunks=False)
        mask = a > 0
        got = x[ht.array(mask, split=split)]
        assert_array_equal(got, a[mask], check_split_chunks=False)
        idx = rng.integers(0, a.shape[0], 4)
        assert_array_equal(x[ht.array(idx)], a[idx], check_split_chunks=False)
        # owner-computes assignment of a broadcast value into a slice
        y = x.copy()
        b = a.copy()
        y[key] = 7
        b[key] = 7
        assert_array_equal(y, b)


def check_random_linalg_matmul():
    rng = np.random.default_rng(505)
    for _ in range(8):
        m, k, n = (int(v) for v in rng.integers(1, 9, 3))
        a = rng.standard_normal((m, k))
        b = rng.standard_normal((k, n))
        for sa in (None, 0, 1):
            sb = [None, 0, 1][int(rng.integers(0, 3))]
            c = ht.matmul(ht.array(a, split=sa), ht.array(b, split=sb))
            assert_array_equal(c, a @ b, rtol=1e-9, atol=1e-9, check_split_chunks=False)
        t = ht.array(a, split=int(rng.integers(0, 2)))
        assert_array_equal(ht.linalg.transpose(t), a.T, check_split_chunks=False)
        if m >= k:
            q, r = ht.linalg.qr(ht.array(a, split=0), mode="reduced")
            qn, rn = q.numpy(), r.numpy()
            assert qn.shape == (m, k) and rn.shape == (k, k)
            assert np.allclose(qn @ rn, a, atol=1e-8)
            assert np.allclose(qn.T @ qn, np.eye(k), atol=1e-8)


def check_random_statistics():
    cases, rng = _cases(606, float_only=True)
    for a, split in cases:
        x = ht.array(a, split=split)
        ax = int(rng.integers(0, a.ndim))
        q = float(rng.uniform(0, 100))
        assert_array_equal(ht.percentile(x, q, axis=ax), np.percentile(a, q, axis=ax), rtol=1e-5, atol=1e-5,
                           check_split_chunks=False)
        assert_array_equal(ht.median(x, axis=ax), np.median(a, axis=ax), rtol=1e-5, atol=1e-5,
                           check_split_chunks=False)
        assert_array_equal(ht.cumsum(x, axis=ax), np.cumsum(a, axis=ax), rtol=1e-4, atol=1e-4,
                           check_split_chunks=False)
        assert_array_equal(ht.std(x, axis=ax), np.std(a, axis=ax), rtol=1e-4, atol=1e-5, check_split_chunks=False)


def _tmpdir():
    import tempfile

    comm = ht.MPI_WORLD
    return comm.bcast(tempfile.mkdtemp() if comm.rank == 0 else None, root=0)


def check_random_io_roundtrips():
    """Random shapes / dtypes written from one split and read back into another, through the
    built-in HDF5 writer (contiguous, and chunked with random chunk shapes + deflate / shuffle /
    fletcher32 filters), NetCDF, .npy and CSV - every rank writes its slab in parallel."""
    import os

    comm = ht.MPI_WORLD
    d = _tmpdir()
    rng = np.random.default_rng(707)
    for case in range(8):
        nd = int(rng.integers(1, 4))
        shape = tuple(int(v) for v in rng.integers(1, 9, nd))
        kind = rng.choice(["f", "d", "i"])
        a = (rng.standard_normal(shape) * 10).astype({"f": np.float32, "d": np.float64, "i": np.int32}[kind])
        if kind == "i":
            a = rng.integers(-1000, 1000, shape).astype(np.int32)
        ws = None if rng.random() < 0.25 else int(rng.integers(0, nd))
        rs = None if rng.random() < 0.25 else int(rng.integers(0, nd))
        x = ht.array(a, split=ws)
        h5 = os.path.join(d, "r{}.h5".format(case))
        ht.save_hdf5(x, h5, "plain")
        kw = {"chunks": tuple(int(rng.integers(1, s + 1)) for s in shape)}
        if rng.random() < 0.7:
            kw["compression"] = "gzip"
            kw["compression_opts"] = int(rng.integers(1, 10))
        kw["shuffle"] = bool(rng.random() < 0.5)
        kw["fletcher32"] = bool(rng.random() < 0.5)
        ht.save_hdf5(x, h5, "chunked", mode="a", **kw)
        for name in ("plain", "chunked"):
            y = ht.load_hdf5(h5, name, dtype=x.dtype, split=rs)
            assert y.split == rs and y.dtype == x.dtype, (name, y.split, y.dtype)
            assert_array_equal(y, a)
        nc = os.path.join(d, "r{}.nc".format(case))
        ht.save(x, nc, "v")
        assert_array_equal(ht.load(nc, "v", dtype=x.dtype, split=rs), a)
        npy = os.path.join(d, "r{}.npy".format(case))
        ht.save(x, npy)
        assert_array_equal(ht.load(npy, split=rs), a)
        if nd == 2 and kind != "i":
            csv = os.path.join(d, "r{}.csv".format(case))
            ht.save_csv(x, csv, decimals=9)
            got = ht.load_csv(csv, dtype=ht.float64, split=rs if rs in (None, 0) else 0)
            assert_array_equal(got, a.astype(np.float64), rtol=1e-5, atol=1e-5)
    comm.Barrier()


def check_random_resplit_chain():
    """A random chain of resplits / balances / redistributions keeps values and the chunking rule."""
    rng = np.random.default_rng(808)
    for _ in range(6):
        nd = int(rng.integers(1, 4))
        shape = tuple(int(v) for v in rng.integers(1, 10, nd))
        a = rng.standard_normal(shape)
        x = ht.array(a, split=int(rng.integers(0, nd)))
        for _ in range(4):
            op = rng.choice(["resplit", "balance", "unbalance", "none"])
            if op == "resplit":
                x = ht.resplit(x, None if rng.random() < 0.2 else int(rng.integers(0, nd)))
            elif op == "balance" and x.split is not None:
                x = x.balance()
            elif op == "unbalance" and x.split is not None and x.shape[x.split] > 1:
                # slicing along the split axis leaves the blocks unbalanced (not rebalanced)
                k = int(rng.integers(1, x.shape[x.split] + 1))
                key = [slice(None)] * nd
                key[x.split] = slice(0, k)
                x = x[tuple(key)]
                sl = [slice(None)] * nd
                sl[x.split] = slice(0, k)
                a = a[tuple(sl)]
            assert_array_equal(x, a, check_split_chunks=bool(x.balanced))
        assert abs(float(ht.sum(x)) - float(a.sum())) < 1e-8 * (1 + np.abs(a).sum())


def check_random_linalg_misc():
    """norms, dot / vecdot / outer, trace, tril / triu, cov on random layouts."""
    rng = np.random.default_rng(909)
    for _ in range(8):
        m, n = (int(v) for v in rng.integers(1, 9, 2))
        a = rng.standard_normal((m, n))
        s = None if rng.random() < 0.25 else int(rng.integers(0, 2))
        x = ht.array(a, split=s)
        assert abs(float(ht.linalg.norm(x)) - np.linalg.norm(a)) < 1e-10 * (1 + np.linalg.norm(a))
        assert_array_equal(ht.linalg.vector_norm(x, axis=1), np.linalg.norm(a, axis=1), rtol=1e-10, atol=1e-12,
                           check_split_chunks=False)
        assert_array_equal(ht.linalg.vector_norm(x, axis=0, ord=1), np.abs(a).sum(0), rtol=1e-10, atol=1e-12,
                           check_split_chunks=False)
        assert abs(float(ht.linalg.matrix_norm(x, ord="fro")) - np.linalg.norm(a, "fro")) < 1e-9
        assert abs(float(ht.linalg.matrix_norm(x, ord=1)) - np.linalg.norm(a, 1)) < 1e-9 * (1 + np.abs(a).sum())
        k = int(rng.integers(-3, 4))
        assert_array_equal(ht.tril(x, k), np.tril(a, k), check_split_chunks=False)
        assert_array_equal(ht.triu(x, k), np.triu(a, k), check_split_chunks=False)
        assert abs(float(ht.trace(x)) - np.trace(a)) < 1e-10 * (1 + np.abs(a).sum())
        u = rng.standard_normal(m)
        v = rng.standard_normal(n)
        su = None if rng.random() < 0.3 else 0
        sv = None if rng.random() < 0.3 else 0
        assert_array_equal(ht.outer(ht.array(u, split=su), ht.array(v, split=sv)), np.outer(u, v), rtol=1e-12,
                           atol=1e-12, check_split_chunks=False)
        assert abs(float(ht.dot(ht.array(u, split=su), ht.array(u, split=su))) - u @ u) < 1e-10 * (1 + u @ u)
        if m > 1 and n > 1:
            assert_array_equal(ht.cov(ht.array(a.T.copy(), split=s)), np.cov(a.T), rtol=1e-8, atol=1e-10,
                               check_split_chunks=False)


def check_random_logical_and_sets():
    """any / all / isclose / allclose / unique / nonzero on random layouts (incl. empty results)."""
    cases, rng = _cases(1010)
    for a, split in cases:
        x = ht.array(a, split=split)
        ax = int(rng.integers(0, a.ndim))
        thr = float(rng.uniform(-1.5, 1.5))
        assert bool(ht.any(x > thr)) == bool(np.any(a > thr))
        assert bool(ht.all(x > thr)) == bool(np.all(a > thr))
        assert_array_equal(ht.any(x > thr, axis=ax), np.any(a > thr, axis=ax), check_split_chunks=False)
        assert_array_equal(ht.all(x > thr, axis=ax), np.all(a > thr, axis=ax), check_split_chunks=False)
        b = a + (1e-9 if a.dtype.kind == "f" else 0)
        assert bool(ht.allclose(x, ht.array(b, split=split)))
        assert_array_equal(ht.isclose(x, ht.array(b, split=split)), np.isclose(a, b), check_split_chunks=False)
        r = np.round(a).astype(np.int64)
        u = ht.unique(ht.array(r, split=split), sorted=True)
        assert_array_equal(u, np.unique(r), check_split_chunks=False)
        nz = ht.nonzero(x > thr)
        ref = np.stack(np.nonzero(a > thr), axis=1) if a.ndim > 1 else np.nonzero(a > thr)[0][:, None]
        got = nz.numpy().reshape(-1, a.ndim) if a.ndim > 1 else nz.numpy().reshape(-1, 1)
        assert got.shape == ref.shape and np.array_equal(got, ref), (got, ref)
