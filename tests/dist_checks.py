"""
Check functions that run identically in a world of one (in-process) and in N gloo ranks
(``tests/_dist.py``). Every check builds the same global data on all ranks, distributes it along
every admissible split axis and compares against NumPy / PyTorch on the gathered result (the
reference's ``assert_func_equal`` strategy, ``heat/core/tests/test_suites/basic_test.py:142-306``).
"""
from __future__ import annotations

import os
import numpy as np
import torch

import heat_amd as ht


def _rng(seed=0):
    return np.random.default_rng(seed)


def assert_array_equal(a: ht.DNDarray, expected, rtol=1e-5, atol=1e-6, check_split_chunks=True):
    """Global shape + local chunk + values (after gathering) against a NumPy array."""
    expected = np.asarray(expected)
    if expected.shape == () and tuple(a.gshape) == (1,):
        # full reductions (sum/prod/min/max/argmin/any/...) have shape (1,) like the reference's
        # (_operations.py:416-417), where NumPy returns a scalar
        expected = expected.reshape(1)
    assert tuple(a.gshape) == tuple(expected.shape), "shape {} != {}".format(a.gshape, expected.shape)
    if check_split_chunks and a.split is not None and a.balanced:
        _, lshape, _ = a.comm.chunk(a.gshape, a.split)
        assert tuple(a.lshape) == tuple(lshape), "local shape {} != chunk {}".format(a.lshape, lshape)
    got = a.numpy()
    if expected.dtype.kind in "fc" or got.dtype.kind in "fc":
        assert np.allclose(got, expected, rtol=rtol, atol=atol, equal_nan=True), "values differ:\n{}\n{}".format(
            got, expected)
    else:
        assert np.array_equal(got, expected), "values differ:\n{}\n{}".format(got, expected)


def for_splits(data: np.ndarray):
    yield None
    for s in range(data.ndim):
        yield s


# ---------------------------------------------------------------------------------------------
def check_basic_plumbing():
    x = ht.arange(10, split=0)
    s = ht.sum(x)
    assert s.item() == 45
    assert x.dtype == ht.int32
    y = ht.arange(10, split=0).astype(ht.float32)
    assert abs(ht.mean(y).item() - 4.5) < 1e-6
    assert x.lshape == x.comm.chunk((10,), 0)[1]


def check_elementwise():
    rng = _rng(1)
    a = rng.standard_normal((7, 5)).astype(np.float32)
    b = rng.standard_normal((7, 5)).astype(np.float32)
    for s in for_splits(a):
        A = ht.array(a, split=s)
        B = ht.array(b, split=s)
        assert_array_equal(A + B, a + b)
        assert_array_equal(A - 2, a - 2)
        assert_array_equal(3 * A, 3 * a)
        assert_array_equal(A / (np.abs(b) + 1), a / (np.abs(b) + 1))
        assert_array_equal(ht.exp(A), np.exp(a), rtol=1e-5)
        assert_array_equal(ht.sin(A), np.sin(a), rtol=1e-5)
        assert_array_equal(ht.abs(A), np.abs(a))
        assert_array_equal(A > B, a > b)
        assert_array_equal(ht.clip(A, -0.5, 0.5), np.clip(a, -0.5, 0.5))
        assert_array_equal(ht.floor(A), np.floor(a))
        assert_array_equal(A ** 2, a ** 2, rtol=1e-5)
        assert_array_equal(ht.where(A > 0, A, B), np.where(a > 0, a, b))
    # broadcasting with a replicated row vector
    row = rng.standard_normal((5,)).astype(np.float32)
    for s in (None, 0, 1):
        assert_array_equal(ht.array(a, split=s) * ht.array(row), a * row)
    # different splits are aligned automatically
    assert_array_equal(ht.array(a, split=0) + ht.array(b, split=1), a + b)


def check_reductions():
    rng = _rng(2)
    a = rng.standard_normal((9, 4, 3)).astype(np.float64)
    for s in for_splits(a):
        A = ht.array(a, split=s)
        assert_array_equal(ht.sum(A), a.sum())
        for ax in range(3):
            assert_array_equal(ht.sum(A, axis=ax), a.sum(axis=ax))
            assert_array_equal(ht.max(A, axis=ax), a.max(axis=ax))
            assert_array_equal(ht.min(A, axis=ax), a.min(axis=ax))
            assert_array_equal(ht.mean(A, axis=ax), a.mean(axis=ax))
            assert_array_equal(ht.var(A, axis=ax), a.var(axis=ax))
            assert_array_equal(ht.std(A, axis=ax, ddof=1), a.std(axis=ax, ddof=1))
            assert_array_equal(ht.argmax(A, axis=ax), a.argmax(axis=ax))
            assert_array_equal(ht.argmin(A, axis=ax), a.argmin(axis=ax))
            assert_array_equal(ht.prod(A, axis=ax), a.prod(axis=ax))
            assert_array_equal(ht.cumsum(A, axis=ax), a.cumsum(axis=ax))
        assert_array_equal(ht.sum(A, axis=(0, 2)), a.sum(axis=(0, 2)))
        assert_array_equal(ht.mean(A, axis=(0, 2)), a.mean(axis=(0, 2)))
        assert_array_equal(ht.mean(A), a.mean())
        assert_array_equal(ht.var(A), a.var())
        assert ht.argmax(A).item() == a.argmax()
        assert ht.argmin(A).item() == a.argmin()
        assert ht.all(A > -100).item() and not ht.any(A > 100).item()
    b = (rng.random((10,)) > 0.5)
    for s in (None, 0):
        assert_array_equal(ht.all(ht.array(b, split=s)), b.all())
        assert_array_equal(ht.any(ht.array(b, split=s)), b.any())


def check_moments_higher():
    rng = _rng(3)
    a = rng.standard_normal((50, 6))
    from scipy import stats

    for s in for_splits(a):
        A = ht.array(a, split=s)
        assert_array_equal(ht.skew(A, axis=0, unbiased=False), stats.skew(a, axis=0, bias=True), rtol=1e-6)
        assert_array_equal(ht.kurtosis(A, axis=0, unbiased=False), stats.kurtosis(a, axis=0, bias=True), rtol=1e-6)
        assert_array_equal(ht.skew(A, axis=1, unbiased=True), stats.skew(a, axis=1, bias=False), rtol=1e-6)
        assert_array_equal(ht.median(A, axis=0), np.median(a, axis=0))
        assert_array_equal(ht.median(A), np.median(a))
        assert_array_equal(ht.percentile(A, [10, 50, 90], axis=1), np.percentile(a, [10, 50, 90], axis=1))
        assert_array_equal(ht.cov(A), np.cov(a), rtol=1e-6)
        assert_array_equal(ht.average(A, axis=0, weights=ht.array(np.arange(50) + 1.0)),
                           np.average(a, axis=0, weights=np.arange(50) + 1.0))


def check_manipulations():
    rng = _rng(4)
    a = rng.integers(-50, 50, size=(8, 6)).astype(np.int64)
    for s in for_splits(a):
        A = ht.array(a, split=s)
        assert_array_equal(ht.reshape(A, (6, 8)), a.reshape(6, 8))
        assert_array_equal(ht.reshape(A, (4, 2, 6)), a.reshape(4, 2, 6))
        assert_array_equal(ht.flatten(A), a.flatten())
        assert_array_equal(ht.flip(A, 0), np.flip(a, 0))
        assert_array_equal(ht.flip(A, 1), np.flip(a, 1))
        assert_array_equal(ht.roll(A, 3, 0), np.roll(a, 3, 0))
        assert_array_equal(ht.roll(A, -2, 1), np.roll(a, -2, 1))
        assert_array_equal(ht.roll(A, 5), np.roll(a, 5))
        assert_array_equal(ht.transpose(A), a.T)
        assert_array_equal(ht.concatenate([A, A], axis=0), np.concatenate([a, a], axis=0))
        assert_array_equal(ht.concatenate([A, A], axis=1), np.concatenate([a, a], axis=1))
        assert_array_equal(ht.stack([A, A], axis=1), np.stack([a, a], axis=1))
        assert_array_equal(ht.pad(A, ((1, 2), (0, 3)), constant_values=7), np.pad(a, ((1, 2), (0, 3)), constant_values=7))
        assert_array_equal(ht.tile(A, (2, 1)), np.tile(a, (2, 1)))
        assert_array_equal(ht.tile(A, (1, 3)), np.tile(a, (1, 3)))
        assert_array_equal(ht.repeat(A, 2, axis=0), np.repeat(a, 2, axis=0))
        assert_array_equal(ht.rot90(A), np.rot90(a))
        assert_array_equal(ht.expand_dims(A, 1), np.expand_dims(a, 1))
        assert_array_equal(ht.squeeze(ht.expand_dims(A, 0)), a)
        assert_array_equal(ht.diagonal(A), np.diagonal(a))
        assert_array_equal(ht.diagonal(A, offset=2), np.diagonal(a, offset=2))
        assert_array_equal(ht.resplit(A, 0), a)
        assert_array_equal(ht.resplit(A, 1), a)
        assert_array_equal(ht.resplit(A, None), a)
        vals, idx = ht.sort(A, axis=0)
        assert_array_equal(vals, np.sort(a, axis=0))
        vals, idx = ht.sort(A, axis=1, descending=True)
        assert_array_equal(vals, -np.sort(-a, axis=1))
        parts = ht.split(A, 2, axis=0)
        for p, e in zip(parts, np.split(a, 2, axis=0)):
            assert_array_equal(p, e, check_split_chunks=False)
        u = ht.unique(A, sorted=True)
        assert_array_equal(u, np.unique(a))
        v, i = ht.topk(A, 2, dim=0)
        assert_array_equal(v, -np.sort(-a, axis=0)[:2])
    v = rng.standard_normal(17)
    for s in (None, 0):
        V = ht.array(v, split=s)
        vs, vi = ht.sort(V)
        assert_array_equal(vs, np.sort(v))
        assert_array_equal(vi, np.argsort(v, kind="stable"))
        assert_array_equal(ht.diag(V), np.diag(v))
        assert_array_equal(ht.hstack([V, V]), np.hstack([v, v]))
        assert_array_equal(ht.vstack([V, V]), np.vstack([v, v]))
        assert_array_equal(ht.diff(V), np.diff(v))
        assert_array_equal(ht.diff(V, n=2), np.diff(v, n=2))


def check_indexing():
    rng = _rng(5)
    a = rng.standard_normal((11, 4))
    for s in for_splits(a):
        A = ht.array(a, split=s)
        assert_array_equal(A[3], a[3])
        assert_array_equal(A[-1], a[-1])
        assert_array_equal(A[2:9], a[2:9], check_split_chunks=False)
        assert_array_equal(A[1:10:3], a[1:10:3], check_split_chunks=False)
        assert_array_equal(A[:, 1], a[:, 1], check_split_chunks=False)
        assert_array_equal(A[::-1], a[::-1], check_split_chunks=False)
        assert_array_equal(A[[5, 0, 7]], a[[5, 0, 7]], check_split_chunks=False)
        assert_array_equal(A[A > 0.5], a[a > 0.5], check_split_chunks=False)
        assert_array_equal(A[2, 3], a[2, 3])
        B = ht.array(a, split=s)
        B[2] = 7.0
        c = a.copy()
        c[2] = 7.0
        assert_array_equal(B, c)
        B[1:5, 2] = ht.array(np.arange(4.0))
        c[1:5, 2] = np.arange(4.0)
        assert_array_equal(B, c)
        B[B > 1.0] = -1.0
        c[c > 1.0] = -1.0
        assert_array_equal(B, c)
        B[[0, 10]] = 3.0
        c[[0, 10]] = 3.0
        assert_array_equal(B, c)
        nz = ht.nonzero(ht.array(a > 0.8, split=s))
        assert_array_equal(nz, np.argwhere(a > 0.8), check_split_chunks=False)


def check_linalg():
    rng = _rng(6)
    a = rng.standard_normal((9, 7))
    b = rng.standard_normal((7, 5))
    v = rng.standard_normal(7)
    for sa in (None, 0, 1):
        for sb in (None, 0, 1):
            A = ht.array(a, split=sa)
            B = ht.array(b, split=sb)
            assert_array_equal(A @ B, a @ b, rtol=1e-6, check_split_chunks=False)
        V = ht.array(v, split=0 if sa is not None else None)
        assert_array_equal(ht.matmul(ht.array(a, split=sa), V), a @ v, rtol=1e-6, check_split_chunks=False)
        assert abs(ht.dot(V, V).item() - v @ v) < 1e-9
    for s in (None, 0, 1):
        A = ht.array(a, split=s)
        assert_array_equal(ht.tril(A), np.tril(a))
        assert_array_equal(ht.triu(A, 1), np.triu(a, 1))
        assert abs(ht.norm(A).item() - np.linalg.norm(a)) < 1e-9
        assert_array_equal(ht.linalg.matrix_norm(A, ord=1), np.linalg.norm(a, ord=1))
        assert_array_equal(ht.linalg.vector_norm(A, axis=0), np.linalg.norm(a, axis=0))
        assert abs(ht.trace(A) - np.trace(a)) < 1e-9
        assert_array_equal(ht.outer(ht.array(v, split=s if s == 0 else None), ht.array(v)), np.outer(v, v))
    tall = rng.standard_normal((40, 6))
    for s in (None, 0, 1):
        q, r = ht.linalg.qr(ht.array(tall, split=s))
        assert_array_equal(q @ r, tall, rtol=1e-6, atol=1e-8, check_split_chunks=False)
        q2, r2 = ht.linalg.qr(ht.array(tall, split=s), mode="reduced")
        qq = q2.numpy()
        assert np.allclose(qq.T @ qq, np.eye(6), atol=1e-8)
        assert np.allclose(qq @ r2.numpy(), tall, atol=1e-8)
    spd = tall.T @ tall + np.eye(6)
    x0 = ht.zeros(6, split=0)
    sol = ht.linalg.cg(ht.array(spd, split=0), ht.array(np.ones(6), split=0), x0)
    assert np.allclose(sol.numpy(), np.linalg.solve(spd, np.ones(6)), atol=1e-6)
    V, T = ht.lanczos(ht.array(spd, split=0), 6)
    vv = V.numpy()
    assert np.allclose(vv.T @ vv, np.eye(6), atol=1e-6)
    assert np.allclose(np.sort(np.linalg.eigvalsh(T.numpy())), np.sort(np.linalg.eigvalsh(spd)), rtol=1e-5)


def check_random():
    ht.random.seed(12345)
    a = ht.random.rand(2, 50, split=0)
    ht.random.seed(12345)
    b = ht.random.rand(100, split=None)
    assert np.array_equal(a.numpy().flatten(), b.numpy())
    ht.random.set_state(("Threefry", 12345, 0xFFFFFFFFFFFFFFF0))
    a = ht.random.rand(2, 3, 4, 5, split=0).numpy().flatten()
    ht.random.set_state(("Threefry", 12345, 0x10000000000000000))
    b = ht.random.rand(2, 44, split=0).numpy().flatten()
    assert np.array_equal(a[32:], b)
    ht.random.seed(12345)
    a = ht.random.rand(2, 34, split=0).numpy().flatten()
    ht.random.set_state(("Threefry", 12345, 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF0))
    b = ht.random.rand(2, 50, split=0).numpy().flatten()
    assert np.array_equal(a, b[32:])
    ht.random.seed(5)
    x = ht.random.randn(4000, split=0)
    assert abs(ht.mean(x).item()) < 0.1 and abs(ht.std(x).item() - 1) < 0.1
    r = ht.random.randint(3, 9, size=(100,), split=0).numpy()
    assert r.min() >= 3 and r.max() < 9
    p = ht.random.permutation(ht.arange(20, split=0)).numpy()
    assert sorted(p.tolist()) == list(range(20))
    st = ht.random.get_state()
    u = ht.random.rand(7).numpy()
    ht.random.set_state(st)
    assert np.array_equal(u, ht.random.rand(7).numpy())


def check_spatial_cluster():
    rng = _rng(7)
    x = rng.standard_normal((30, 4)).astype(np.float32)
    y = rng.standard_normal((20, 4)).astype(np.float32)
    from scipy.spatial.distance import cdist as scd

    for sx in (None, 0):
        for sy in (None, 0):
            X, Y = ht.array(x, split=sx), ht.array(y, split=sy)
            d = ht.spatial.cdist(X, Y)
            assert_array_equal(d, scd(x, y), rtol=1e-4, atol=1e-4, check_split_chunks=False)
            assert_array_equal(ht.spatial.manhattan(X, Y), scd(x, y, "cityblock"), rtol=1e-4, atol=1e-4,
                               check_split_chunks=False)
            assert_array_equal(ht.spatial.rbf(X, Y, sigma=2.0), np.exp(-scd(x, y, "sqeuclidean") / 8.0), rtol=1e-4,
                               atol=1e-5, check_split_chunks=False)
    centers = np.array([[0, 0], [8, 8], [-8, 8]], dtype=np.float32)
    pts = np.concatenate([c + rng.standard_normal((60, 2)).astype(np.float32) for c in centers])
    for s in (None, 0):
        X = ht.array(pts, split=s)
        for Est in (ht.cluster.KMeans, ht.cluster.KMedians, ht.cluster.KMedoids):
            est = Est(n_clusters=3, init="kmeans++", random_state=1) if Est is not ht.cluster.KMeans else \
                Est(n_clusters=3, init="kmeans++", random_state=1, max_iter=100)
            est.fit(X)
            got = est.cluster_centers_.numpy()
            dist = scd(got, centers).min(axis=1)
            assert np.all(dist < 1.0), (Est.__name__, got)
            lab = est.predict(X).numpy().reshape(-1)
            assert lab.shape == (180,)


def check_io_csv():
    import os
    import tempfile

    comm = ht.MPI_WORLD
    data = np.arange(60, dtype=np.float64).reshape(20, 3) / 7
    path = os.path.join(tempfile.gettempdir(), "heat_amd_io_{}.csv".format(os.getpid() if comm.size == 1 else "mp"))
    if comm.rank == 0:
        np.savetxt(path, data, delimiter=",", header="a,b,c", comments="")
    comm.Barrier()
    for s in (None, 0):
        x = ht.load_csv(path, header_lines=1, split=s, dtype=ht.float64)
        assert_array_equal(x, data)
    p2 = path + ".npy"
    X = ht.array(data, split=0)
    ht.save(X, p2)
    y = ht.load(p2, split=0)
    assert_array_equal(y, data)
    comm.Barrier()


# ---------------------------------------------------------------------------------------------
# estimators / nn / data (reference: heat/regression/lasso/tests, heat/naive_bayes/tests,
# heat/classification/tests, heat/nn/tests, heat/optim/tests, heat/utils/data/tests)
# ---------------------------------------------------------------------------------------------
def _blobs(n_per, centers, seed=0, scale=0.3):
    rng = _rng(seed)
    X = np.concatenate([rng.normal(c, scale, size=(n_per, len(c))) for c in centers]).astype(np.float32)
    y = np.repeat(np.arange(len(centers)), n_per)
    return X, y


def check_lasso():
    rng = _rng(3)
    m, n = 240, 6
    X = rng.normal(size=(m, n)).astype(np.float32)
    X[:, 0] = 1.0
    X /= np.sqrt((X ** 2).mean(0))          # the reference's update assumes unit mean-square columns
    w = np.array([0.5, 2.0, 0.0, -1.5, 0.0, 0.7], np.float32)
    y = (X @ w + 0.01 * rng.normal(size=m)).astype(np.float32)
    thetas = []
    prev = os.environ.get("HEAT_LASSO_SOLVER")
    for split, solver in ((None, "sweep"), (0, "sweep"), (None, "gram"), (0, "gram")):
        os.environ["HEAT_LASSO_SOLVER"] = solver
        try:
            est = ht.regression.Lasso(lam=0.01, max_iter=200, tol=1e-7)
            est.fit(ht.array(X, split=split), ht.array(y[:, None], split=split))
        finally:
            if prev is None:
                os.environ.pop("HEAT_LASSO_SOLVER", None)
            else:
                os.environ["HEAT_LASSO_SOLVER"] = prev
        th = est.theta.numpy().ravel()
        thetas.append(th)
        pred = est.predict(ht.array(X, split=split)).numpy().ravel()
        assert np.sqrt(np.mean((pred - y) ** 2)) < 0.05
    for t in thetas[1:]:
        assert np.allclose(thetas[0], t, atol=1e-4)
    assert abs(thetas[0][2]) < 0.02 and abs(thetas[0][4]) < 0.02       # sparsity of the zero weights
    assert np.allclose(thetas[0], w, atol=0.05)


def check_gaussian_nb():
    from sklearn.naive_bayes import GaussianNB as SkNB

    X, y = _blobs(40, [(0, 0, 0), (2, 2, 0), (0, 3, 3)], seed=5, scale=0.8)
    sk = SkNB().fit(X, y)
    for split in (None, 0):
        nb = ht.naive_bayes.GaussianNB()
        nb.fit(ht.array(X, split=split), ht.array(y, split=split))
        assert np.allclose(nb.theta_.numpy(), sk.theta_, atol=1e-4)
        assert np.allclose(nb.var_.numpy() if hasattr(nb, "var_") else nb.sigma_.numpy(), sk.var_, rtol=1e-3,
                           atol=1e-5)
        pred = nb.predict(ht.array(X, split=split)).numpy()
        assert np.array_equal(pred, sk.predict(X))
        proba = nb.predict_proba(ht.array(X, split=split)).numpy()
        assert np.allclose(proba, sk.predict_proba(X), atol=1e-4)


def check_knn():
    from sklearn.neighbors import KNeighborsClassifier as SkKNN

    X, y = _blobs(30, [(0, 0), (3, 0), (0, 3)], seed=7, scale=1.0)
    Q = _rng(8).normal(1.0, 1.5, size=(25, 2)).astype(np.float32)
    sk = SkKNN(n_neighbors=5).fit(X, y)
    for split in (None, 0):
        knn = ht.classification.KNeighborsClassifier(n_neighbors=5)
        knn.fit(ht.array(X, split=split), ht.array(y, split=split))
        pred = knn.predict(ht.array(Q, split=split)).numpy().ravel()
        assert (pred == sk.predict(Q)).mean() > 0.95


def check_kmedians_kmedoids_spectral():
    X, y = _blobs(30, [(0, 0), (6, 6), (-6, 6)], seed=9, scale=0.5)
    for cls in (ht.cluster.KMedians, ht.cluster.KMedoids):
        est = cls(n_clusters=3, init="kmeans++", random_state=1)
        labels = est.fit_predict(ht.array(X, split=0)).numpy().ravel()
        for c in range(3):
            assert len(np.unique(labels[y == c])) == 1
        assert len(np.unique(labels)) == 3
    sp = ht.cluster.Spectral(n_clusters=3, gamma=0.5, metric="rbf", laplacian="fully_connected", n_lanczos=40)
    labels = sp.fit_predict(ht.array(X, split=0)).numpy().ravel()
    assert len(np.unique(labels)) == 3
    for c in range(3):
        assert len(np.unique(labels[y == c])) == 1


def check_data_parallel():
    comm = ht.MPI_WORLD
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.ReLU(), torch.nn.Linear(8, 1))
    opt = ht.optim.DataParallelOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), blocking=True)
    dp = ht.nn.DataParallel(net, comm, opt, blocking_parameter_updates=True, bucket_cap_mb=0.0001)
    ref = torch.nn.Sequential(torch.nn.Linear(4, 8), torch.nn.ReLU(), torch.nn.Linear(8, 1))
    ref.load_state_dict(net.state_dict())
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(1)
    per = 6
    for _ in range(3):
        Xg = torch.randn(per * comm.size, 4, generator=g)
        yg = torch.randn(per * comm.size, 1, generator=g)
        Xl, yl = Xg[comm.rank * per:(comm.rank + 1) * per], yg[comm.rank * per:(comm.rank + 1) * per]
        opt.zero_grad()
        torch.nn.functional.mse_loss(dp(Xl), yl).backward()
        opt.step()
        ref_opt.zero_grad()
        torch.nn.functional.mse_loss(ref(Xg), yg).backward()
        ref_opt.step()
    for p, q in zip(net.parameters(), ref.parameters()):
        assert torch.allclose(p, q, atol=1e-5), (p, q)


def check_dataloader_shuffle():
    comm = ht.MPI_WORLD
    n = 8 * comm.size          # Dataset keeps gshape // size rows per rank (reference semantics)
    data = ht.array(np.arange(n * 2, dtype=np.float32).reshape(n, 2), split=0)
    ds = ht.utils.data.Dataset(data)
    loader = ht.utils.data.DataLoader(ds, batch_size=4)
    for _epoch in range(3):
        seen = torch.cat([b for b in loader]) if len(loader) else torch.empty(0, 2)
        assert seen.shape[0] == data.lshape[0]
        allrows = np.concatenate(comm.allgather(seen.cpu().numpy()))
        assert sorted(allrows[:, 0].tolist()) == list(np.arange(0, 2 * n, 2, dtype=np.float32))


def check_tiling():
    a = ht.zeros((7, 5, 6), split=1)
    t = ht.tiling.SplitTiles(a)
    assert tuple(t.tile_dimensions.sum(dim=1).tolist()) == (7, 5, 6)
    assert t.tile_locations.shape == (a.comm.size,) * 3
    m = ht.zeros((12, 9), split=0)
    sq = ht.tiling.SquareDiagTiles(m, tiles_per_proc=2)
    assert sum(sq.row_indices[i + 1] - sq.row_indices[i] for i in range(len(sq.row_indices) - 1)) <= 12
    assert sq.tile_rows >= 2


# ---------------------------------------------------------------------------------------------
# communication layer, one check per primitive family (reference heat/core/tests/
# test_communication.py: blocking + non-blocking, IN_PLACE, axis permutations, v-variants)
# ---------------------------------------------------------------------------------------------
def check_comm_collectives():
    comm = ht.MPI_WORLD
    p, me = comm.size, comm.rank
    MPI = ht.MPI
    # Bcast / Ibcast
    t = torch.full((3, 2), float(me))
    comm.Bcast(t, root=p - 1)
    assert torch.all(t == p - 1)
    t = torch.arange(4.0) * (me + 1)
    comm.Ibcast(t, root=0).Wait()
    assert torch.equal(t, torch.arange(4.0))
    # Allreduce with every op, IN_PLACE and separate buffers, blocking and not
    vals = [torch.tensor([r + 1.0, -(r + 2.0), 2.0 ** r]) for r in range(p)]
    mine = vals[me]
    expect = {MPI.SUM: sum(vals), MPI.PROD: torch.stack(vals).prod(0), MPI.MAX: torch.stack(vals).max(0).values,
              MPI.MIN: torch.stack(vals).min(0).values}
    for op, ref in expect.items():
        out = torch.empty(3)
        comm.Allreduce(mine, out, op)
        assert torch.allclose(out, ref), (op, out, ref)
        buf = mine.clone()
        comm.Iallreduce(MPI.IN_PLACE, buf, op).Wait()
        assert torch.allclose(buf, ref)
    bits = torch.tensor([1 << me, 7], dtype=torch.int64)
    comm.Allreduce(MPI.IN_PLACE, bits, MPI.BOR)
    assert int(bits[0]) == (1 << p) - 1 and int(bits[1]) == 7
    flags = torch.tensor([True, me == 0])
    comm.Allreduce(MPI.IN_PLACE, flags, MPI.LAND)
    assert bool(flags[0]) and bool(flags[1]) == (p == 1)
    flags = torch.tensor([False, me == 0])
    comm.Allreduce(MPI.IN_PLACE, flags, MPI.LOR)
    assert not bool(flags[0]) and bool(flags[1])
    custom = MPI.Op.Create(lambda a, b, *args: torch.maximum(a, b) + 0 * b)
    buf = torch.tensor([float(me)])
    comm.Allreduce(MPI.IN_PLACE, buf, custom)
    assert float(buf) == p - 1
    # Exscan / Scan
    s = torch.tensor([float(me + 1)])
    ex = torch.zeros(1)
    comm.Exscan(s, ex, MPI.SUM)
    if me > 0:
        assert float(ex) == sum(range(1, me + 1))
    sc = torch.zeros(1)
    comm.Scan(s, sc, MPI.SUM)
    assert float(sc) == sum(range(1, me + 2))
    # Allgather along axis 0 and 1 (equal counts)
    blk = torch.full((2, 3), float(me))
    out = torch.empty((2 * p, 3))
    comm.Allgather(blk, out, recv_axis=0)
    assert torch.equal(out, torch.cat([torch.full((2, 3), float(r)) for r in range(p)], 0))
    out = torch.empty((2, 3 * p))
    comm.Iallgather(blk, out, recv_axis=1).Wait()
    assert torch.equal(out, torch.cat([torch.full((2, 3), float(r)) for r in range(p)], 1))
    # Allgatherv with uneven counts + IN_PLACE
    counts = [r + 1 for r in range(p)]
    displs = [sum(counts[:r]) for r in range(p)]
    send = torch.full((counts[me], 2), float(me))
    recv = torch.empty((sum(counts), 2))
    comm.Allgatherv(send, (recv, counts, displs))
    assert torch.equal(recv, torch.cat([torch.full((c, 2), float(r)) for r, c in enumerate(counts)]))
    recv2 = torch.zeros((sum(counts), 2))
    recv2[displs[me]: displs[me] + counts[me]] = float(me)
    comm.Allgatherv(MPI.IN_PLACE, (recv2, counts, displs))
    assert torch.equal(recv2, recv)
    # Gatherv / Scatterv
    g = torch.empty((sum(counts), 2)) if me == 0 else None
    comm.Gatherv(send, (g, counts, displs) if me == 0 else None, root=0)
    if me == 0:
        assert torch.equal(g, recv)
    sc_out = torch.empty((counts[me], 2))
    comm.Scatterv((recv, counts, displs) if me == 0 else None, sc_out, root=0)
    assert torch.all(sc_out == float(me))
    # Alltoall (equal) and Alltoallv (uneven) along axis 0 and 1
    a2 = torch.arange(p * 2, dtype=torch.float32).reshape(p * 2, 1) + 100 * me
    r2 = torch.empty_like(a2)
    comm.Alltoall(a2, r2)
    expect = torch.cat([torch.arange(2 * me, 2 * me + 2, dtype=torch.float32).reshape(2, 1) + 100 * r
                        for r in range(p)])
    assert torch.equal(r2, expect)
    a3 = a2.t().contiguous()
    r3 = torch.empty_like(a3)
    comm.Alltoall(a3, r3, send_axis=1)
    assert torch.equal(r3, expect.t())
    scounts = [(me + r) % 2 + 1 for r in range(p)]
    rcounts = [(r + me) % 2 + 1 for r in range(p)]
    sv = torch.cat([torch.full((scounts[r],), float(100 * me + r)) for r in range(p)])
    rv = torch.empty(sum(rcounts))
    comm.Alltoallv((sv, scounts), (rv, rcounts))
    assert torch.equal(rv, torch.cat([torch.full((rcounts[r],), float(100 * r + me)) for r in range(p)]))
    # point to point ring: Send/Recv and Isend/Irecv
    if p > 1:
        nxt, prv = (me + 1) % p, (me - 1) % p
        got = torch.empty(3)
        if me % 2 == 0:
            comm.Send(torch.full((3,), float(me)), nxt)
            comm.Recv(got, prv)
        else:
            comm.Recv(got, prv)
            comm.Send(torch.full((3,), float(me)), nxt)
        assert torch.all(got == prv)
        rq = comm.Irecv(got, prv)
        sq = comm.Isend(torch.full((3,), float(me + 10)), nxt)
        sq.Wait()
        rq.Wait()
        assert torch.all(got == prv + 10)
    # pickled object collectives
    assert comm.bcast({"a": me}, root=0) == {"a": 0}
    assert comm.allgather(me) == list(range(p))
    assert comm.allreduce(me + 1) == p * (p + 1) // 2
    assert comm.alltoall([me * 10 + r for r in range(p)]) == [r * 10 + me for r in range(p)]
    gathered = comm.gather(me, root=0)
    assert (gathered == list(range(p))) if me == 0 else gathered is None
    assert comm.scatter([r * r for r in range(p)] if me == 0 else None, root=0) == me * me
    # sub-communicators
    sub = comm.Split(color=me % 2, key=-me)
    members = [r for r in range(p) if r % 2 == me % 2]
    assert sub.size == len(members)
    assert sub.rank == sorted(members, reverse=True).index(me)
    tot = torch.tensor([float(me)])
    sub.Allreduce(MPI.IN_PLACE, tot, MPI.SUM)
    assert float(tot) == sum(members)
    x = ht.arange(10, split=0, comm=sub)
    assert int(ht.sum(x).item()) == 45
    comm.Barrier()


def check_daso():
    """DASO end to end (reference optim/tests/test_dp_optimizer.py, which needs 8 GPUs): warm-up,
    skipping phase with stale global averages, cool-down; afterwards every rank holds the same
    parameters and the loss went down. Even world sizes run as nodes of 2 ranks."""
    import os

    comm = ht.MPI_WORLD
    old = os.environ.get("LOCAL_WORLD_SIZE")
    os.environ["LOCAL_WORLD_SIZE"] = "2" if comm.size % 2 == 0 else "1"
    try:
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.Tanh(), torch.nn.Linear(16, 1))
        opt = torch.optim.SGD(net.parameters(), lr=0.05)
        daso = ht.optim.DASO(local_optimizer=opt, total_epochs=6, comm=comm, warmup_epochs=1, cooldown_epochs=1,
                             max_global_skips=4, stability_level=0.5)
        dp = ht.nn.DataParallelMultiGPU(net, daso, comm)
        g = torch.Generator().manual_seed(10 + comm.rank)
        w_true = torch.linspace(-1, 1, 6)
        X = torch.randn(96, 6, generator=g)
        y = (X @ w_true).unsqueeze(1)
        nb = 12
        daso.last_batch = nb - 1
        losses = []
        for epoch in range(6):
            tot = 0.0
            for b in range(nb):
                xb, yb = X[b * 8:(b + 1) * 8], y[b * 8:(b + 1) * 8]
                daso.zero_grad()
                loss = torch.nn.functional.mse_loss(dp(xb), yb)
                loss.backward()
                daso.step()
                tot += float(loss)
            losses.append(tot / nb)
            daso.epoch_loss_logic(torch.tensor(tot / nb))
        flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()])
        allp = comm.allgather(flat.numpy())
        for other in allp[1:]:
            assert np.allclose(other, allp[0], atol=1e-6)
        assert losses[-1] < losses[0]
    finally:
        if old is None:
            os.environ.pop("LOCAL_WORLD_SIZE", None)
        else:
            os.environ["LOCAL_WORLD_SIZE"] = old


def check_custom_reduction_ops():
    """Packed (value, index) and top-k reduction callbacks (reference MPI_ARGMAX / MPI_TOPK)."""
    from heat_amd.core import manipulations, statistics

    comm = ht.MPI_WORLD
    p, me = comm.size, comm.rank
    vals = torch.tensor([float((me * 7) % 5), float(me)], dtype=torch.float64)
    idx = torch.tensor([float(me * 10), float(me * 10 + 1)], dtype=torch.float64)
    buf = torch.cat([vals, idx])
    comm.Allreduce(ht.MPI.IN_PLACE, buf, statistics.MPI_ARGMAX)
    allv = [((r * 7) % 5, r * 10) for r in range(p)]
    best = max(allv, key=lambda t: (t[0], -t[1]))
    assert float(buf[0]) == best[0] and float(buf[2]) == best[1]
    assert float(buf[1]) == p - 1 and float(buf[3]) == (p - 1) * 10 + 1
    buf = torch.cat([vals, idx])
    comm.Allreduce(ht.MPI.IN_PLACE, buf, statistics.MPI_ARGMIN)
    worst = min(allv, key=lambda t: (t[0], t[1]))
    assert float(buf[0]) == worst[0] and float(buf[2]) == worst[1]
    # top-2 along dim 0 of per-rank candidates
    k = 2
    cand = torch.tensor([[float(me), float(-me)], [float(me + 0.5), float(-me - 0.5)]], dtype=torch.float64)
    cidx = torch.tensor([[me * 2.0, me * 2.0], [me * 2.0 + 1, me * 2.0 + 1]], dtype=torch.float64)
    meta = torch.tensor([k, 0, 1, 1, 2, 2, 2], dtype=torch.float64)
    buf = torch.cat([meta, cand.flatten(), cidx.flatten()])
    comm.Allreduce(ht.MPI.IN_PLACE, buf, manipulations.MPI_TOPK)
    res = buf[7: 7 + 4].reshape(2, 2)
    allc = torch.cat([torch.tensor([[float(r), float(-r)], [r + 0.5, -r - 0.5]], dtype=torch.float64)
                      for r in range(p)])
    ref = torch.topk(allc, k, dim=0).values
    # a one-rank reduction never calls the operator (MPI semantics): compare the sets
    assert torch.equal(res.sort(0, descending=True).values, ref)


def check_io_hdf5_netcdf():
    """HDF5 / netCDF round trips on every split (parallel slab writes), and reads of the
    reference's own h5py / netCDF-4 fixtures when the reference tree is present."""
    import os
    import tempfile

    comm = ht.MPI_WORLD
    d = comm.bcast(tempfile.mkdtemp() if comm.rank == 0 else None, root=0)
    data = np.arange(7 * 5, dtype=np.float32).reshape(7, 5) / 3.0
    for split in (None, 0, 1):
        x = ht.array(data, split=split)
        ht.save_hdf5(x, os.path.join(d, "a.h5"), "data")
        ht.save_hdf5(x.astype(ht.int64), os.path.join(d, "a.h5"), "ints", mode="a")
        for rsplit in (None, 0, 1):
            y = ht.load(os.path.join(d, "a.h5"), "data", split=rsplit)
            assert_array_equal(y, data)
            z = ht.load_hdf5(os.path.join(d, "a.h5"), "ints", dtype=ht.int64, split=rsplit)
            assert_array_equal(z, data.astype(np.int64))
        ht.save(x, os.path.join(d, "a.nc"), "var")
        for rsplit in (None, 0, 1):
            assert_array_equal(ht.load(os.path.join(d, "a.nc"), "var", split=rsplit), data)
    part = ht.load_hdf5(os.path.join(d, "a.h5"), "data", split=0, load_fraction=0.5)
    assert part.shape == (3, 5)
    ref = "/root/reference/heat/datasets"
    if os.path.isdir(ref):
        iris_csv = ht.load_csv(os.path.join(ref, "iris.csv"), sep=";", split=0)
        assert ht.allclose(ht.load(os.path.join(ref, "iris.h5"), "data", split=0), iris_csv)
        assert ht.allclose(ht.load(os.path.join(ref, "iris.nc"), "data", split=1), iris_csv)
        xd = ht.load_hdf5(os.path.join(ref, "diabetes.h5"), "x", split=0)
        assert xd.shape == (442, 11)
    comm.Barrier()


def check_partial_h5_dataset():
    """PartialH5Dataset streams this rank's share of an HDF5 file window by window
    (reference utils/data/tests/test_partial_dataset.py)."""
    import os
    import tempfile

    comm = ht.MPI_WORLD
    d = comm.bcast(tempfile.mkdtemp() if comm.rank == 0 else None, root=0)
    n = 40 * comm.size
    data = np.arange(n * 3, dtype=np.float32).reshape(n, 3)
    labels = np.arange(n, dtype=np.float32)
    path = os.path.join(d, "p.h5")
    ht.save_hdf5(ht.array(data, split=0), path, "data")
    ht.save_hdf5(ht.array(labels, split=0), path, "labels", mode="a")
    ds = ht.utils.data.PartialH5Dataset(path, comm=comm, dataset_names=["data", "labels"], use_gpu=False,
                                        initial_load=16, load_length=8)
    loader = ht.utils.data.DataLoader(ds, batch_size=4)
    seen = []
    for x, y in loader:
        assert torch.equal(x[:, 0] / 3, y)
        seen.append(y)
    got = torch.cat(seen).sort().values
    lo = comm.rank * (n // comm.size)
    assert got.numel() >= 16 and float(got.min()) >= lo and float(got.max()) < lo + n // comm.size


def check_collective_guard():
    """A failure on one rank surfaces on every rank (no deadlock in the next collective)."""
    from heat_amd.parallel import RemoteRankError, collective_guard

    comm = ht.MPI_WORLD
    raised = None
    try:
        with collective_guard(comm):
            if comm.rank == comm.size - 1:
                raise ValueError("bad input on the last rank")
    except ValueError:
        raised = "own"
    except RemoteRankError as e:
        raised = "remote"
        assert e.rank == comm.size - 1
    assert raised == ("own" if comm.rank == comm.size - 1 else "remote")
    with collective_guard(comm):
        pass
    assert int(ht.sum(ht.arange(10, split=0)).item()) == 45  # the world is still usable


def check_getitem_setitem_semantics():
    """Split propagation and local shapes of __getitem__/__setitem__ (the reference's rules,
    heat/core/dndarray.py:661-1549; cases from its bug reports #730/#825)."""
    comm = ht.MPI_WORLD
    p = comm.size
    # assigning a smaller split array into an interior window
    for split, win, setshape in ((0, (slice(1, -1), slice(1, -1)), (100, 100)),
                                 (1, (slice(-30, None), slice(1, -1)), (30, 100)),
                                 (1, (slice(1, -1), slice(None, 20)), (100, 20))):
        a = ht.ones((102, 102), split=split)
        a[win] = ht.zeros(setshape, split=split)
        assert bool(ht.all(a[win] == 0))
        ref = np.ones((102, 102), np.float32)
        ref[win] = 0
        assert_array_equal(a, ref, check_split_chunks=False)
    # split of a result after integer indexing
    a = ht.ones((10, 25, 30), split=1)
    if p > 1:
        assert a[0].split == 0
        assert a[:, 0, :].split is None
        assert a[:, :, 0].split == 1
    # scalar get / set, numpy and torch integer keys
    a = ht.zeros((13, 5), split=0)
    a[10, np.array(0)] = 1
    assert float(a[10, 0].item()) == 1 and a[10, 0].dtype == ht.float32
    a = ht.zeros((13, 5), split=0)
    a[10] = 1
    b = a[torch.tensor(10)]
    assert bool((b == 1).all()) and b.gshape == (5,) and b.dtype == ht.float32
    a[-1] = 2
    assert bool((a[-1] == 2).all())
    # slices keep the split and are not rebalanced
    a = ht.zeros((13, 5), split=0)
    a[1:4] = 1
    s_ = a[1:4]
    assert bool((s_ == 1).all()) and s_.gshape == (3, 5) and s_.split == 0
    counts = a.comm.counts_displs_shape((13, 5), 0)[0]
    lo = sum(counts[: comm.rank])
    mine = max(0, min(lo + counts[comm.rank], 4) - max(lo, 1))
    assert s_.lshape == (mine, 5)
    b = a[1:4, np.int64(1)]
    assert b.gshape == (3,) and b.split == 0 and bool((b == 1).all())
    c = ht.zeros((13, 5), split=0)
    c[8:12, ht.array(1)] = 1
    b = c[8:12, np.int64(1)]
    assert b.gshape == (4,) and b.split == 0 and bool((b == 1).all())
    # boolean mask keeps the split axis, values equal numpy
    data = np.arange(24, dtype=np.float32).reshape(6, 4)
    for split in (None, 0, 1):
        x = ht.array(data, split=split)
        m = x > 10
        got = x[m]
        assert np.array_equal(np.sort(got.numpy()), data[data > 10])
        x[m] = -1
        ref = data.copy()
        ref[ref > 10] = -1
        assert_array_equal(x, ref, check_split_chunks=False)
    # advanced (list) indexing along the split axis and step slices
    for split in (None, 0, 1):
        x = ht.array(data, split=split)
        assert_array_equal(x[[4, 0, 5]], data[[4, 0, 5]], check_split_chunks=False)
        assert_array_equal(x[::-2], data[::-2], check_split_chunks=False)
        assert_array_equal(x[1:5:2, ::3], data[1:5:2, ::3], check_split_chunks=False)
        assert_array_equal(x[..., 1], data[..., 1], check_split_chunks=False)
        assert_array_equal(x[None, 2], data[None, 2], check_split_chunks=False)


def check_manipulations_more():
    """The remaining manipulation / statistics functions against NumPy on every split axis."""
    rng = _rng(21)
    a3 = rng.normal(size=(4, 6, 5)).astype(np.float32)
    a2 = rng.normal(size=(6, 4)).astype(np.float32)
    v = rng.normal(size=(6,)).astype(np.float32)
    for split in for_splits(a3):
        x = ht.array(a3, split=split)
        assert_array_equal(ht.moveaxis(x, 0, -1), np.moveaxis(a3, 0, -1), check_split_chunks=False)
        assert_array_equal(ht.swapaxes(x, 0, 2), np.swapaxes(a3, 0, 2), check_split_chunks=False)
        assert_array_equal(ht.rot90(x, 1, (0, 1)), np.rot90(a3, 1, (0, 1)), check_split_chunks=False)
        assert_array_equal(ht.rot90(x, -1, (1, 2)), np.rot90(a3, -1, (1, 2)), check_split_chunks=False)
        assert_array_equal(ht.ravel(x), np.ravel(a3), check_split_chunks=False)
        for got, ref in zip(ht.dsplit(x, 5), np.dsplit(a3, 5)):
            assert_array_equal(got, ref, check_split_chunks=False)
        for got, ref in zip(ht.hsplit(x, [2, 5]), np.hsplit(a3, [2, 5])):
            assert_array_equal(got, ref, check_split_chunks=False)
        for got, ref in zip(ht.vsplit(x, 2), np.vsplit(a3, 2)):
            assert_array_equal(got, ref, check_split_chunks=False)
        assert ht.shape(x) == a3.shape
    for split in for_splits(a2):
        x = ht.array(a2, split=split)
        assert_array_equal(ht.fliplr(x), np.fliplr(a2), check_split_chunks=False)
        assert_array_equal(ht.flipud(x), np.flipud(a2), check_split_chunks=False)
        y = ht.array(a2 * 2, split=split)
        assert_array_equal(ht.maximum(x, y), np.maximum(a2, a2 * 2), check_split_chunks=False)
        assert_array_equal(ht.minimum(x, y), np.minimum(a2, a2 * 2), check_split_chunks=False)
        vs = ht.array(v, split=0 if split is not None else None)
        assert_array_equal(ht.column_stack((x, vs)), np.column_stack((a2, v)), check_split_chunks=False)
        assert_array_equal(ht.row_stack((x, x)), np.vstack((a2, a2)), check_split_chunks=False)
    ints = rng.integers(0, 7, size=50)
    for split in (None, 0):
        xi = ht.array(ints, split=split)
        assert_array_equal(ht.bincount(xi), np.bincount(ints))
        w = ht.array(np.linspace(0, 1, 50, dtype=np.float32), split=split)
        assert_array_equal(ht.bincount(xi, weights=w, minlength=10),
                           np.bincount(ints, weights=np.linspace(0, 1, 50, dtype=np.float32), minlength=10),
                           rtol=1e-5)
        xf = ht.array(ints.astype(np.float32), split=split)
        h = ht.histc(xf, bins=7, min=0, max=7)
        assert_array_equal(h, np.histogram(ints, bins=7, range=(0, 7))[0].astype(np.float32))


def check_sort_batched():
    """Sample sort of many columns at once along every split axis: values, stable global indices
    (ties), descending order, integer / bool keys and ranks without rows; median/percentile."""
    rng = _rng(33)
    a = rng.integers(0, 5, size=(7, 3, 11)).astype(np.int64)  # many ties
    f = rng.normal(size=(7, 3, 11)).astype(np.float32)
    for split in for_splits(a):
        for axis in range(3):
            x = ht.array(a, split=split)
            v, i = ht.sort(x, axis=axis)
            assert_array_equal(v, np.sort(a, axis=axis, kind="stable"))
            assert_array_equal(i, np.argsort(a, axis=axis, kind="stable"))
            v, i = ht.sort(x, axis=axis, descending=True)
            assert_array_equal(v, -np.sort(-a, axis=axis, kind="stable"))
            assert_array_equal(i, np.argsort(-a, axis=axis, kind="stable"))
            y = ht.array(f, split=split)
            v, i = ht.sort(y, axis=axis, descending=True)
            assert_array_equal(v, -np.sort(-f, axis=axis))
            assert_array_equal(ht.median(y, axis=axis), np.median(f, axis=axis), check_split_chunks=False)
            assert_array_equal(ht.percentile(y, [10.0, 75.0], axis=axis),
                               np.percentile(f, [10.0, 75.0], axis=axis), check_split_chunks=False)
        b = ht.array(a > 2, split=split)
        v, i = ht.sort(b, axis=0)
        assert_array_equal(v, np.sort(a > 2, axis=0, kind="stable"))
        assert_array_equal(i, np.argsort(a > 2, axis=0, kind="stable"))
    short = rng.normal(size=(2, 4)).astype(np.float32)  # fewer rows than ranks (p = 3)
    v, i = ht.sort(ht.array(short, split=0), axis=0)
    assert_array_equal(v, np.sort(short, axis=0))
    assert_array_equal(i, np.argsort(short, axis=0, kind="stable"))


def check_printing():
    """``str(DNDarray)`` matches the reference's format (printed on rank 0 only)."""
    import math

    comm = ht.MPI_WORLD
    try:
        s = str(ht.array([], dtype=ht.int64, device="cpu"))
        assert comm.rank != 0 or s == "DNDarray([], dtype=ht.int64, device=cpu:0, split=None)"
        s = str(ht.array(42, device="cpu"))
        assert comm.rank != 0 or s == "DNDarray(42, dtype=ht.int64, device=cpu:0, split=None)"
        s = str(ht.arange(2 * 3 * 4, device="cpu").reshape((2, 3, 4)))
        assert comm.rank != 0 or s == ("DNDarray([[[ 0,  1,  2,  3],\n           [ 4,  5,  6,  7],\n"
                                       "           [ 8,  9, 10, 11]],\n\n          [[12, 13, 14, 15],\n"
                                       "           [16, 17, 18, 19],\n           [20, 21, 22, 23]]], dtype=ht.int32, "
                                       "device=cpu:0, split=None)")
        s = str(ht.arange(12 * 13 * 14, split=0, device="cpu").reshape((12, 13, 14)))
        if comm.rank == 0:
            assert s.startswith("DNDarray([[[   0,    1,    2,  ...,   11,   12,   13],\n")
            assert s.endswith("[2170, 2171, 2172,  ..., 2181, 2182, 2183]]], dtype=ht.int32, device=cpu:0, "
                              "split=0)")
        ht.set_printoptions(precision=2)
        s = str(ht.arange(0.5, 2 * 3 * 4 + 0.5, split=0, device="cpu").reshape((2, 3, 4)))
        assert comm.rank != 0 or "[20.50, 21.50, 22.50, 23.50]]], dtype=ht.float32, device=cpu:0, split=0)" in s
        ht.set_printoptions(profile="full")
        assert ht.get_printoptions()["threshold"] == math.inf
        ht.set_printoptions(profile="short")
        assert ht.get_printoptions()["precision"] == 2 and ht.get_printoptions()["edgeitems"] == 2
    finally:
        ht.set_printoptions(profile="default")


def check_random_counter_semantics():
    """Threefry stream properties (reference core/tests/test_random.py): reseeding reproduces,
    consecutive calls differ, 64-bit counter overflow continues the stream, a 128-bit overflow
    wraps to the beginning, and values do not depend on shape / split / process count."""
    seed = 12345
    ht.random.seed(seed)
    a = ht.random.rand(2, 5, 7, 3, split=0)
    assert a.dtype == ht.float32 and a.larray.dtype == torch.float32
    b = ht.random.rand(2, 5, 7, 3, split=0)
    assert not bool(ht.equal(a, b))
    ht.random.seed(seed)
    assert bool(ht.equal(a, ht.random.rand(2, 5, 7, 3, dtype=ht.float32, split=0)))
    ht.random.set_state(("Threefry", seed, 0xFFFFFFFFFFFFFFF0))
    a = ht.random.rand(2, 3, 4, 5, split=0).numpy().ravel()
    ht.random.set_state(("Threefry", seed, 0x10000000000000000))
    b = ht.random.rand(2, 44, split=0).numpy().ravel()
    assert a.dtype == np.float32 and np.array_equal(a[32:], b)
    ht.random.set_state(("Threefry", seed, 0x100000000))
    a = ht.random.rand(2, 44)
    ht.random.seed(seed)
    assert not bool(ht.equal(a, ht.random.rand(2, 44)))
    ht.random.seed(seed)
    a = ht.random.rand(2, 34, split=0).numpy().ravel()
    ht.random.set_state(("Threefry", seed, 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFF0))
    b = ht.random.rand(2, 50, split=0).numpy().ravel()
    assert np.array_equal(a, b[32:])
    ht.random.seed(seed)
    a = ht.random.rand(2, 50, split=0).numpy().ravel()
    ht.random.seed(seed)
    assert np.array_equal(a, ht.random.rand(100, split=None).numpy())
    ht.random.seed(seed)
    a = ht.random.randn(3, 5, 2, 9, split=3)
    ht.random.seed(seed)
    assert bool(ht.equal(a, ht.random.randn(3, 5, 2, 9, split=3)))
    ht.random.seed(seed)
    ri = ht.random.randint(-5, 9, (40,), split=0, dtype=ht.int64).numpy()
    assert ri.min() >= -5 and ri.max() < 9
    p = ht.random.permutation(30)
    assert sorted(p.numpy().tolist()) == list(range(30))


def check_dndarray_properties():
    """DNDarray attributes and helpers (reference core/tests/test_dndarray.py)."""
    comm = ht.MPI_WORLD
    p, me = comm.size, comm.rank
    # halos along a column split
    data_np = np.arange(1, 3 * 2 * p + 1, dtype=np.float32).reshape(2, 3 * p)
    x = ht.array(data_np, split=1)
    x.get_halo(2)
    counts, displs = x.counts_displs()
    if p > 1:
        if me < p - 1:
            nxt = data_np[:, displs[me + 1]: displs[me + 1] + 2]
            assert np.array_equal(x.halo_next.cpu().numpy(), nxt)
        else:
            assert x.halo_next is None
        if me > 0:
            prv = data_np[:, displs[me] - 2: displs[me]]
            assert np.array_equal(x.halo_prev.cpu().numpy(), prv)
        else:
            assert x.halo_prev is None
        extra = (2 if me > 0 else 0) + (2 if me < p - 1 else 0)
        assert tuple(x.array_with_halos.shape) == (2, counts[me] + extra)
    for bad, exc in (("wrong", TypeError), (-99, ValueError)):
        try:
            x.get_halo(bad)
            raise AssertionError("expected {}".format(exc))
        except exc:
            pass
    # metadata
    y = ht.zeros((7, 4, 3), split=1, dtype=ht.float64)
    assert y.gnumel == 84 and y.size == 84 and y.ndim == 3 and len(y) == 7
    assert y.nbytes == y.gnbytes == 84 * 8
    assert y.lnbytes == y.larray.numel() * 8
    assert y.lnumel == y.larray.numel()
    c, d = y.counts_displs()
    assert sum(c) == 4 and list(d) == [sum(c[:r]) for r in range(p)]
    assert tuple(y.lshape_map[:, 1].tolist()) == tuple(c)
    assert y.is_balanced() and y.balanced
    assert y.is_distributed() == (p > 1)
    assert y.stride() == y.larray.stride() and len(y.strides) == 3
    # item / casts / tolist / numpy
    z = ht.array([[3.5]], split=0)
    assert z.item() == 3.5 and float(z) == 3.5 and int(z) == 3 and bool(z) and complex(z) == 3.5 + 0j
    assert ht.array([[1, 2], [3, 4]], split=0).tolist() == [[1, 2], [3, 4]]
    a = ht.arange(10, split=0)
    assert a.astype(ht.float64).dtype == ht.float64 and a.astype(ht.float64, copy=False).dtype == ht.float64
    # lloc: local indexing
    loc = a.lloc[0:1]
    assert tuple(loc.shape) == (min(1, a.lshape[0]),)
    # fill_diagonal on a split matrix
    m = ht.zeros((5, 5), split=0)
    m.fill_diagonal(2)
    assert_array_equal(m, np.eye(5, dtype=np.float32) * 2)
    # unbalanced -> balance, redistribute, lshape_map
    b = ht.arange(3 * p + 2, split=0)[2:]
    b.balance_()
    assert b.is_balanced()
    assert_array_equal(b, np.arange(2, 3 * p + 2))
    if p > 1:
        target = torch.tensor([[3 * p - 2 * (p - 1)] + [2] * (p - 1)]).T if False else None
        tm = b.lshape_map.clone()
        tm[:, 0] = torch.tensor([3 * p - (p - 1)] + [1] * (p - 1))
        b.redistribute_(lshape_map=b.lshape_map, target_map=tm)
        assert b.lshape[0] == int(tm[me, 0])
        assert_array_equal(b, np.arange(2, 3 * p + 2), check_split_chunks=False)
    # bitwise dunders
    i1 = ht.array([0b1100, 0b1010], split=0)
    i2 = ht.array([0b1010, 0b0110], split=0)
    assert (i1 & i2).tolist() == [8, 2] and (i1 | i2).tolist() == [14, 14] and (i1 ^ i2).tolist() == [6, 12]
    assert (~i1).tolist() == [~12, ~10] and (i1 << 1).tolist() == [24, 20] and (i1 >> 2).tolist() == [3, 2]


def check_linalg_more():
    """Norms with every ord, vecdot, projection, transpose axes, trace offsets, batched matmul."""
    rng = _rng(31)
    a = rng.standard_normal((8, 6))
    b3 = rng.standard_normal((3, 8, 6))
    u, w = rng.standard_normal(6), rng.standard_normal(6)
    for s in (None, 0, 1):
        A = ht.array(a, split=s)
        for o in (1, -1, 2, -2, np.inf, -np.inf, "fro", "nuc"):
            got = float(ht.linalg.matrix_norm(A, ord=o).item())
            assert abs(got - np.linalg.norm(a, ord=o)) < 1e-8 * max(1.0, abs(got)), (o, got)
        for o in (None, 1, 3, np.inf, -np.inf, 0):
            for ax in (0, 1):
                assert_array_equal(ht.linalg.vector_norm(A, axis=ax, ord=o), np.linalg.norm(a, axis=ax, ord=o),
                                   rtol=1e-7, check_split_chunks=False)
        assert_array_equal(ht.transpose(A), a.T, check_split_chunks=False)
        assert abs(ht.trace(A, offset=2) - np.trace(a, offset=2)) < 1e-9
        assert_array_equal(ht.linalg.vecdot(A, A, axis=1), (a * a).sum(1), rtol=1e-9, check_split_chunks=False)
    for s in (None, 0, 2):
        B3 = ht.array(b3, split=s)
        assert_array_equal(ht.transpose(B3, (2, 0, 1)), b3.transpose(2, 0, 1), check_split_chunks=False)
    U, W = ht.array(u, split=0), ht.array(w, split=0)
    pr = ht.linalg.projection(U, W)
    assert_array_equal(pr, (u @ w) / (w @ w) * w, rtol=1e-9)
    assert_array_equal(ht.linalg.vecdot(U, W), np.array(u @ w), rtol=1e-9)


def check_lanczos_collectives_per_step():
    """Lanczos issues at most 2 all-reduces per step beyond its matvec (``[w.w, V^T w]`` and
    ``[u.u, u^T A u]``), counted from the collective-path counters over 6 extra steps, and its
    result still matches the eigenvalues; a rank-deficient matrix (exact breakdown) stays
    orthonormal and finite without any host sync in the loop."""
    from heat_amd.core.communication import PATH_COUNTS

    rng = np.random.default_rng(3)
    n = 40
    B = rng.standard_normal((n, n))
    spd = B @ B.T + n * np.eye(n)
    A = ht.array(spd, split=0)
    v0 = ht.array(np.ones(n) / np.sqrt(n), split=0)

    def allreduces(m):
        before = sum(v for k, v in PATH_COUNTS.items() if k.startswith("allreduce"))
        ht.lanczos(A, m, v0=v0)
        return sum(v for k, v in PATH_COUNTS.items() if k.startswith("allreduce")) - before

    x = ht.ones(n, split=0)
    before = sum(v for k, v in PATH_COUNTS.items() if k.startswith("allreduce"))
    ht.matmul(A, x)
    per_matvec = sum(v for k, v in PATH_COUNTS.items() if k.startswith("allreduce")) - before
    per_step = (allreduces(14) - allreduces(8)) / 6.0
    if ht.MPI_WORLD.size > 1:
        assert per_step - per_matvec <= 2.0, (per_step, per_matvec)
    V, T = ht.lanczos(A, n, v0=v0)
    vv = V.numpy()
    assert np.allclose(vv.T @ vv, np.eye(n), atol=1e-4)
    ev = np.sort(np.linalg.eigvalsh(T.numpy().astype(np.float64)))
    assert np.allclose(ev, np.sort(np.linalg.eigvalsh(spd)), rtol=1e-3)
    # rank-2 matrix: beta hits 0 at step 2, the replacement vector keeps V orthonormal
    u = rng.standard_normal((n, 2))
    low = ht.array(u @ u.T, split=0)
    V, T = ht.lanczos(low, 5, v0=v0)
    vv = V.numpy()
    assert np.all(np.isfinite(vv)) and np.all(np.isfinite(T.numpy()))
    assert np.allclose(vv.T @ vv, np.eye(5), atol=1e-3)
