"""
Oracle checks against scikit-learn and SciPy (both importable here, neither used by the package):
the same inputs through ``heat_amd`` and through the library implementation of the same algorithm,
compared to fp64 round-off. Where the reference's tests pin an estimator on one dataset
(``heat/regression/tests/test_lasso.py``, ``heat/cluster/tests/test_kmeans.py``,
``heat/spatial/tests/test_distances.py``, ``heat/core/tests/test_statistics.py``), these pin it on
seeded random problems, for every split the estimator accepts.

* Lasso: the reference's update ``theta_j = S(rho_j, lam)`` (``heat/regression/lasso.py:152-165``)
  is exact coordinate minimisation of ``1/(2m)|y - X theta|^2 + lam |theta_1:|_1`` when every
  column has mean square 1, so on column-normalised data it has sklearn's ``Lasso`` (intercept
  fitted, not penalised) as its fixed point - both solvers (``gram``, ``sweep``).
* KMeans: Lloyd's algorithm from the same explicit initial centres is deterministic, so centres and
  labels equal sklearn's ``KMeans(algorithm="lloyd", n_init=1)``.
* cdist / rbf / manhattan: ``scipy.spatial.distance.cdist`` on every split pairing.
* skew / kurtosis / percentile / cov: ``scipy.stats`` and NumPy, biased and unbiased.
* KMedians / KMedoids: a NumPy transcription of the reference's L1 Lloyd iteration.
* GaussianNB (fit, weighted fit, partial_fit, probabilities) and KNN votes: sklearn.
* float32 inputs (the native kernels' dtype on the GPU) at fp32 tolerances.

Run in a world of one (``test_core_local.py``) and at 2-8 gloo ranks (``test_distributed.py``).
"""
from __future__ import annotations

import os

import numpy as np

import heat_amd as ht

from .dist_checks import assert_array_equal


def _split_choices(nd):
    return [None] + list(range(nd))


class _env:
    """Temporarily set one environment variable (restored on exit)."""

    def __init__(self, key, value):
        self.key, self.value = key, value

    def __enter__(self):
        self.old = os.environ.get(self.key)
        os.environ[self.key] = self.value

    def __exit__(self, *exc):
        if self.old is None:
            os.environ.pop(self.key, None)
        else:
            os.environ[self.key] = self.old


def _lasso_problem(seed, m, n):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((m, n))
    X /= np.sqrt((X ** 2).mean(axis=0))          # unit mean square: the reference's update is exact CD
    w = np.zeros(n)
    w[: max(1, n // 2)] = rng.uniform(-3, 3, max(1, n // 2))
    y = X @ w + 0.7 + 0.1 * rng.standard_normal(m)
    return np.hstack([np.ones((m, 1)), X]), y


def check_oracle_lasso_sklearn():
    from sklearn.linear_model import Lasso as SkLasso

    for seed, (m, n) in enumerate([(301, 6), (500, 12), (97, 3)]):
        Xa, y = _lasso_problem(seed, m, n)
        for lam in (0.01, 0.2):
            sk = SkLasso(alpha=lam, fit_intercept=True, tol=1e-14, max_iter=200000).fit(Xa[:, 1:], y)
            ref = np.concatenate([[sk.intercept_], sk.coef_])
            for solver in ("gram", "sweep"):
                for split in (None, 0):
                    with _env("HEAT_LASSO_SOLVER", solver):
                        est = ht.regression.Lasso(lam=lam, max_iter=20000, tol=1e-13)
                        est.fit(ht.array(Xa, split=split), ht.array(y, split=split))
                    th = est.theta.numpy().ravel()
                    err = np.abs(th - ref).max()
                    assert err < 1e-9, (seed, lam, solver, split, err, th, ref)
                    # predictions of the fitted model agree as well
                    pred = est.predict(ht.array(Xa, split=split)).numpy().ravel()
                    np.testing.assert_allclose(pred, sk.predict(Xa[:, 1:]), rtol=1e-9, atol=1e-9)


def _blobs(seed, k, f, per, spread=0.3):
    rng = np.random.default_rng(seed)
    centres = rng.uniform(-10, 10, (k, f))
    pts = np.concatenate([c + spread * rng.standard_normal((per + i, f)) for i, c in enumerate(centres)])
    return pts[rng.permutation(len(pts))], rng


def check_oracle_kmeans_sklearn_lloyd():
    from sklearn.cluster import KMeans as SkKMeans

    for seed, (k, f, per) in enumerate([(4, 3, 40), (7, 5, 25), (3, 2, 60)]):
        X, rng = _blobs(seed, k, f, per, spread=1.5)        # overlapping: Lloyd needs several steps
        init = X[rng.choice(len(X), k, replace=False)]
        for iters in (1, 3, 50):
            sk = SkKMeans(n_clusters=k, init=init, n_init=1, max_iter=iters, tol=0.0, algorithm="lloyd").fit(X)
            for split in (None, 0):
                km = ht.cluster.KMeans(n_clusters=k, init=ht.array(init), max_iter=iters, tol=None)
                km.fit(ht.array(X, split=split))
                c = km.cluster_centers_.numpy()
                np.testing.assert_allclose(c, sk.cluster_centers_, rtol=1e-10, atol=1e-10,
                                           err_msg="seed {} iters {} split {}".format(seed, iters, split))
                lab = km.predict(ht.array(X, split=split)).numpy().ravel()
                np.testing.assert_array_equal(lab, sk.predict(X))


def check_oracle_cdist_scipy():
    from scipy.spatial.distance import cdist as sp_cdist

    rng = np.random.default_rng(7)
    for m, n, f in [(13, 9, 4), (5, 17, 1), (24, 24, 7)]:
        a = rng.standard_normal((m, f))
        b = rng.standard_normal((n, f))
        d2 = sp_cdist(a, b, "sqeuclidean")
        for sa in (None, 0):
            for sb in (None, 0):
                X, Y = ht.array(a, split=sa), ht.array(b, split=sb)
                assert_array_equal(ht.spatial.cdist(X, Y), np.sqrt(d2), rtol=1e-9, atol=1e-9)
                assert_array_equal(ht.spatial.cdist(X, Y, quadratic_expansion=True), np.sqrt(d2),
                                   rtol=1e-7, atol=1e-7)
                assert_array_equal(ht.spatial.manhattan(X, Y), sp_cdist(a, b, "cityblock"), rtol=1e-9, atol=1e-9)
                assert_array_equal(ht.spatial.rbf(X, Y, sigma=1.7), np.exp(-d2 / (2 * 1.7 ** 2)),
                                   rtol=1e-9, atol=1e-9)
        # self-distance: zero diagonal, symmetric
        X = ht.array(a, split=0)
        assert_array_equal(ht.spatial.cdist(X), sp_cdist(a, a), rtol=1e-9, atol=1e-9)


def check_oracle_moments_scipy():
    from scipy import stats

    rng = np.random.default_rng(11)
    for shape in [(40,), (9, 13), (5, 6, 7)]:
        a = rng.gamma(2.0, 1.5, shape)                     # skewed, heavy-ish tail
        for split in _split_choices(a.ndim):
            x = ht.array(a, split=split)
            for axis in [None] + list(range(a.ndim)):
                for unbiased in (True, False):
                    ref_s = stats.skew(a, axis=axis, bias=not unbiased)
                    assert_array_equal(ht.skew(x, axis=axis, unbiased=unbiased), np.asarray(ref_s),
                                       rtol=1e-9, atol=1e-10)
                    for fisher in (True, False):
                        ref_k = stats.kurtosis(a, axis=axis, fisher=fisher, bias=not unbiased)
                        assert_array_equal(ht.kurtosis(x, axis=axis, unbiased=unbiased, Fischer=fisher),
                                           np.asarray(ref_k), rtol=1e-9, atol=1e-10)


def check_oracle_percentile_numpy():
    rng = np.random.default_rng(12)
    methods = ["linear", "lower", "higher", "midpoint", "nearest"]
    for shape in [(31,), (8, 11)]:
        a = rng.standard_normal(shape)
        for split in _split_choices(a.ndim):
            x = ht.array(a, split=split)
            for axis in [None] + list(range(a.ndim)):
                for meth in methods:
                    for q in (0.0, 12.5, 50.0, 99.0, 100.0):
                        ref = np.percentile(a, q, axis=axis, method=meth)
                        got = ht.percentile(x, q, axis=axis, interpolation=meth)
                        assert_array_equal(got, np.asarray(ref), rtol=1e-12, atol=1e-12)
                    qs = [5.0, 50.0, 95.0]
                    got = ht.percentile(x, qs, axis=axis, interpolation=meth)
                    assert_array_equal(got, np.percentile(a, qs, axis=axis, method=meth), rtol=1e-12, atol=1e-12)
            assert_array_equal(ht.median(x, axis=0), np.median(a, axis=0), rtol=1e-12, atol=1e-12)


def check_oracle_cov_numpy():
    rng = np.random.default_rng(13)
    for m, n in [(4, 30), (7, 9), (2, 5)]:
        a = rng.standard_normal((m, n))
        b = rng.standard_normal((m, n))
        for split in (None, 0, 1):
            x = ht.array(a, split=split)
            assert_array_equal(ht.cov(x), np.cov(a), rtol=1e-10, atol=1e-12)
            assert_array_equal(ht.cov(x, bias=True), np.cov(a, bias=True), rtol=1e-10, atol=1e-12)
            assert_array_equal(ht.cov(x, ddof=2), np.cov(a, ddof=2), rtol=1e-10, atol=1e-12)
            xt = ht.array(a.T.copy(), split=split)
            assert_array_equal(ht.cov(xt, rowvar=False), np.cov(a.T, rowvar=False), rtol=1e-10, atol=1e-12)
            assert_array_equal(ht.cov(x, ht.array(b, split=split)), np.cov(a, b), rtol=1e-10, atol=1e-12)


def _l1_lloyd(X, C, iters, medoids):
    """NumPy k-medians / k-medoids (the reference's algorithm, ``heat/cluster/kmedians.py:57-100``,
    ``kmedoids.py:56-114``): L1 assignment, per-cluster coordinate median; k-medoids then moves each
    centre to the sample closest (L1) to that median. Stops when the centres stop moving."""
    C = C.copy()
    for _ in range(iters):
        lab = np.abs(X[:, None, :] - C[None, :, :]).sum(-1).argmin(1)
        new = C.copy()
        for i in range(len(C)):
            pts = X[lab == i]
            if len(pts) == 0:
                continue
            med = np.median(pts, axis=0)
            new[i] = X[np.abs(X - med).sum(1).argmin()] if medoids else med
        if np.array_equal(new, C):
            break
        C = new
    return C, np.abs(X[:, None, :] - C[None, :, :]).sum(-1).argmin(1)


def check_oracle_kmedians_kmedoids_numpy():
    for seed, (k, f, per) in enumerate([(3, 2, 30), (5, 4, 21)]):
        X, rng = _blobs(100 + seed, k, f, per, spread=1.0)
        init = X[rng.choice(len(X), k, replace=False)]
        for est_cls, medoids in ((ht.cluster.KMedians, False), (ht.cluster.KMedoids, True)):
            for iters in (1, 2, 30):
                C_ref, lab_ref = _l1_lloyd(X, init, iters, medoids)
                for split in (None, 0):
                    kw = {} if medoids else {"tol": None}     # KMedoids has no tol (reference API)
                    est = est_cls(n_clusters=k, init=ht.array(init), max_iter=iters, **kw)
                    est.fit(ht.array(X, split=split))
                    np.testing.assert_allclose(est.cluster_centers_.numpy(), C_ref, rtol=1e-12, atol=1e-12,
                                               err_msg="{} seed {} iters {} split {}".format(
                                                   est_cls.__name__, seed, iters, split))
                    np.testing.assert_array_equal(est.predict(ht.array(X, split=split)).numpy().ravel(), lab_ref)


def _nb_var(nb):
    """Per-class variances (``sigma_``, the reference's name; sklearn >= 1.0 calls them ``var_``)."""
    return (nb.var_ if hasattr(nb, "var_") else nb.sigma_).numpy()


def check_oracle_gaussian_nb_sklearn():
    """fp64 GaussianNB against sklearn to round-off: one-shot fit, incremental ``partial_fit`` over
    three batches (the reference's chunked mean/variance merge), sample weights, probabilities."""
    from sklearn.naive_bayes import GaussianNB as SkNB

    rng = np.random.default_rng(21)
    X = np.concatenate([rng.normal(c, 1.0 + 0.2 * i, (35 + 3 * i, 4)) for i, c in enumerate((-2.0, 0.5, 2.5))])
    y = np.repeat(np.arange(3), [35, 38, 41])
    p = rng.permutation(len(y))
    X, y = X[p], y[p]
    w = rng.uniform(0.5, 2.0, len(y))
    sk = SkNB().fit(X, y)
    skw = SkNB().fit(X, y, sample_weight=w)
    skp = SkNB()
    for part in np.array_split(np.arange(len(y)), 3):
        skp.partial_fit(X[part], y[part], classes=np.arange(3))
    for split in (None, 0):
        hx, hy = ht.array(X, split=split), ht.array(y, split=split)
        nb = ht.naive_bayes.GaussianNB().fit(hx, hy)
        np.testing.assert_allclose(nb.theta_.numpy(), sk.theta_, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(_nb_var(nb), sk.var_, rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(nb.class_prior_.numpy(), sk.class_prior_, rtol=1e-12)
        np.testing.assert_array_equal(nb.predict(hx).numpy().ravel(), sk.predict(X))
        np.testing.assert_allclose(nb.predict_proba(hx).numpy(), sk.predict_proba(X), rtol=1e-8, atol=1e-12)
        np.testing.assert_allclose(nb.predict_log_proba(hx).numpy(), sk.predict_log_proba(X), rtol=1e-8, atol=1e-8)
        nbw = ht.naive_bayes.GaussianNB().fit(hx, hy, sample_weight=ht.array(w, split=split))
        np.testing.assert_allclose(nbw.theta_.numpy(), skw.theta_, rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(_nb_var(nbw), skw.var_, rtol=1e-10, atol=1e-12)
        nbp = ht.naive_bayes.GaussianNB()
        for part in np.array_split(np.arange(len(y)), 3):
            nbp.partial_fit(ht.array(X[part], split=split), ht.array(y[part], split=split),
                            classes=ht.array(np.arange(3)))
        np.testing.assert_allclose(nbp.theta_.numpy(), skp.theta_, rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(_nb_var(nbp), skp.var_, rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(nbp.class_count_.numpy(), skp.class_count_)


def check_oracle_knn_sklearn():
    """fp64 k-nearest-neighbour votes equal sklearn's on continuous data (no distance ties) for
    odd k and two classes (no vote ties), every split of the training and query sets."""
    from sklearn.neighbors import KNeighborsClassifier as SkKNN

    rng = np.random.default_rng(22)
    X = np.concatenate([rng.normal(0.0, 1.0, (40, 3)), rng.normal(1.2, 1.0, (45, 3))])
    y = np.repeat([0, 1], [40, 45])
    Q = rng.normal(0.6, 1.3, (33, 3))
    for k in (1, 5, 9):
        ref = SkKNN(n_neighbors=k).fit(X, y).predict(Q)
        for sx in (None, 0):
            for sq in (None, 0):
                knn = ht.classification.KNeighborsClassifier(n_neighbors=k)
                knn.fit(ht.array(X, split=sx), ht.array(y, split=sx))
                np.testing.assert_array_equal(knn.predict(ht.array(Q, split=sq)).numpy().ravel(), ref)


def check_oracle_fp32_paths():
    """float32 inputs - the dtype the native MFMA / VALU kernels take on the GPU - against fp64
    library results, at fp32 tolerances: Lloyd from a fixed init on well-separated blobs (labels
    exact), the exact and expanded distance kernels, both Lasso solvers, mean / var / std."""
    from scipy.spatial.distance import cdist as sp_cdist
    from sklearn.cluster import KMeans as SkKMeans
    from sklearn.linear_model import Lasso as SkLasso

    X, rng = _blobs(31, 6, 8, 50, spread=0.4)
    init = X[rng.choice(len(X), 6, replace=False)]
    sk = SkKMeans(n_clusters=6, init=init, n_init=1, max_iter=20, tol=0.0, algorithm="lloyd").fit(X)
    X32 = X.astype(np.float32)
    for split in (None, 0):
        km = ht.cluster.KMeans(n_clusters=6, init=ht.array(init.astype(np.float32)), max_iter=20, tol=None)
        km.fit(ht.array(X32, split=split))
        np.testing.assert_allclose(km.cluster_centers_.numpy(), sk.cluster_centers_, rtol=2e-5, atol=2e-5)
        np.testing.assert_array_equal(km.predict(ht.array(X32, split=split)).numpy().ravel(), sk.labels_)

    a = rng.standard_normal((70, 19)).astype(np.float32)
    b = rng.standard_normal((45, 19)).astype(np.float32)
    d = sp_cdist(a.astype(np.float64), b.astype(np.float64))
    for split in (None, 0):
        A, B = ht.array(a, split=split), ht.array(b)
        assert_array_equal(ht.spatial.cdist(A, B), d, rtol=1e-5, atol=1e-5)
        assert_array_equal(ht.spatial.cdist(A, B, quadratic_expansion=True), d, rtol=1e-4, atol=1e-4)
        assert_array_equal(ht.spatial.manhattan(A, B), sp_cdist(a.astype(np.float64), b.astype(np.float64),
                                                                "cityblock"), rtol=1e-5, atol=1e-5)

    Xa, y = _lasso_problem(32, 400, 10)
    ref = SkLasso(alpha=0.05, tol=1e-14, max_iter=200000).fit(Xa[:, 1:], y)
    ref = np.concatenate([[ref.intercept_], ref.coef_])
    for solver in ("gram", "sweep"):
        for split in (None, 0):
            with _env("HEAT_LASSO_SOLVER", solver):
                est = ht.regression.Lasso(lam=0.05, max_iter=2000, tol=1e-7)
                est.fit(ht.array(Xa.astype(np.float32), split=split), ht.array(y.astype(np.float32), split=split))
            np.testing.assert_allclose(est.theta.numpy().ravel(), ref, rtol=1e-4, atol=1e-4)

    m = rng.gamma(2.0, 1.0, (300, 17)).astype(np.float32)
    for split in (None, 0, 1):
        x = ht.array(m, split=split)
        for axis in (None, 0, 1):
            assert_array_equal(ht.mean(x, axis=axis), np.asarray(m.astype(np.float64).mean(axis=axis)),
                               rtol=1e-5, atol=1e-6)
            assert_array_equal(ht.var(x, axis=axis, ddof=1), np.asarray(m.astype(np.float64).var(axis=axis, ddof=1)),
                               rtol=1e-4, atol=1e-6)
            assert_array_equal(ht.std(x, axis=axis), np.asarray(m.astype(np.float64).std(axis=axis)),
                               rtol=1e-4, atol=1e-6)


def check_oracle_linalg_numpy():
    """fp64 linear algebra against NumPy/SciPy for every split: matmul (all 9 split pairings),
    QR (R up to row signs, Q orthonormal), singular values, vector / matrix norms of every order,
    conjugate gradients on an SPD system, and Lanczos (T = V^T A V, orthonormal V)."""
    import scipy.linalg as sla

    rng = np.random.default_rng(41)
    a = rng.standard_normal((23, 7))
    b = rng.standard_normal((7, 11))
    for sa in (None, 0, 1):
        for sb in (None, 0, 1):
            assert_array_equal(ht.matmul(ht.array(a, split=sa), ht.array(b, split=sb)), a @ b, rtol=1e-10, atol=1e-10)
    for split in (None, 0, 1):
        x = ht.array(a, split=split)
        q, r = ht.linalg.qr(x, mode="reduced")
        rn = np.linalg.qr(a, mode="r")
        sgn = np.sign(np.diag(r.numpy())) * np.sign(np.diag(rn))
        np.testing.assert_allclose(r.numpy(), sgn[:, None] * rn, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(q.numpy().T @ q.numpy(), np.eye(7), atol=1e-10)
        np.testing.assert_allclose(q.numpy() @ r.numpy(), a, atol=1e-10)
        s = ht.linalg.svd(x, compute_uv=False)
        np.testing.assert_allclose(s.numpy(), np.linalg.svd(a, compute_uv=False), rtol=1e-10, atol=1e-10)
        for ordv in (None, "fro", "nuc", 1, -1, 2, -2, np.inf, -np.inf):
            assert_array_equal(ht.linalg.matrix_norm(x, ord=ordv), np.asarray(np.linalg.norm(a, ord=ordv)),
                               rtol=1e-9, atol=1e-10)
    v = rng.standard_normal(29)
    for split in (None, 0):
        xv = ht.array(v, split=split)
        for ordv in (None, 0, 1, 2, 3, np.inf, -np.inf, 0.5):
            assert_array_equal(ht.linalg.vector_norm(xv, ord=ordv), np.asarray(np.linalg.norm(v, ord=ordv)),
                               rtol=1e-10, atol=1e-10)

    n = 24
    m = rng.standard_normal((n, n))
    A = m @ m.T + n * np.eye(n)                           # SPD, well conditioned
    rhs = rng.standard_normal(n)
    ref = sla.solve(A, rhs, assume_a="pos")
    for split in (None, 0):
        sol = ht.linalg.cg(ht.array(A, split=split), ht.array(rhs, split=split), ht.zeros(n, dtype=ht.float64,
                                                                                           split=split))
        np.testing.assert_allclose(sol.numpy(), ref, rtol=1e-8, atol=1e-8)
        V, T = ht.linalg.lanczos(ht.array(A, split=split), 10, v0=ht.array(np.ones(n) / np.sqrt(n), split=split))
        Vn, Tn = V.numpy(), T.numpy()
        np.testing.assert_allclose(Vn.T @ Vn, np.eye(10), atol=1e-8)
        np.testing.assert_allclose(Vn.T @ A @ Vn, Tn, atol=1e-8)
        # the extreme Ritz values bracket inside the spectrum
        ev, rv = np.linalg.eigvalsh(A), np.linalg.eigvalsh(Tn)
        assert ev[0] - 1e-9 <= rv[0] and rv[-1] <= ev[-1] + 1e-9


def check_oracle_cdist_topk_sklearn():
    """``spatial.cdist_topk`` / ``cdist_argmin`` (fused nearest-neighbour reduction, no distance
    matrix) against sklearn's exact ``NearestNeighbors`` for every split of X and Y, fp64 and fp32;
    exact duplicates in Y check the (distance, index) tie order."""
    from sklearn.neighbors import NearestNeighbors

    rng = np.random.default_rng(51)
    a = rng.standard_normal((37, 6))
    b = rng.standard_normal((29, 6))
    for k in (1, 4, 29):
        nn = NearestNeighbors(n_neighbors=k, algorithm="brute").fit(b)
        ref_d, ref_i = nn.kneighbors(a)
        for sa in (None, 0):
            for sb in (None, 0):
                for dt, tol in ((np.float64, 1e-10), (np.float32, 2e-5)):
                    d, i = ht.spatial.cdist_topk(ht.array(a.astype(dt), split=sa), ht.array(b.astype(dt), split=sb), k)
                    assert d.split == sa and i.split == sa and d.gshape == (37, k)
                    np.testing.assert_allclose(d.numpy(), ref_d, rtol=tol, atol=tol)
                    np.testing.assert_array_equal(i.numpy(), ref_i)
    # exact duplicates (fp64, exact path): equal distances come in index order, on any split
    bd = b.copy()
    bd[7] = bd[3]
    bd[20] = bd[3]
    for sb in (None, 0):
        for k in (1, 2, 3):
            d, i = ht.spatial.cdist_topk(ht.array(bd[3:4] + 1e-3), ht.array(bd, split=sb), k)
            np.testing.assert_array_equal(i.numpy(), [[3, 7, 20][:k]])
            assert np.all(d.numpy() == d.numpy()[0, 0])
    dm, im = ht.spatial.cdist_argmin(ht.array(a, split=0), ht.array(b, split=0))
    ref_d, ref_i = NearestNeighbors(n_neighbors=1, algorithm="brute").fit(b).kneighbors(a)
    np.testing.assert_array_equal(im.numpy(), ref_i[:, 0])
    np.testing.assert_allclose(dm.numpy(), ref_d[:, 0], rtol=1e-10)
    # fewer query rows than ranks (empty local blocks) and a Y smaller than the world
    d3, i3 = ht.spatial.cdist_topk(ht.array(a[:3], split=0), ht.array(b[:2], split=0), 2)
    r3 = NearestNeighbors(n_neighbors=2, algorithm="brute").fit(b[:2]).kneighbors(a[:3])
    np.testing.assert_array_equal(i3.numpy(), r3[1])
    np.testing.assert_allclose(d3.numpy(), r3[0], rtol=1e-10)
    # self-query: every row's nearest neighbour is itself at distance 0
    ds, is_ = ht.spatial.cdist_topk(ht.array(a, split=0), None, 1)
    np.testing.assert_array_equal(is_.numpy()[:, 0], np.arange(37))


def check_cdist_topk_arguments():
    a = ht.array(np.zeros((4, 3)), split=0)
    for bad_k in (0, 5, 1.5):
        try:
            ht.spatial.cdist_topk(a, a, bad_k)
        except ValueError:
            pass
        else:
            raise AssertionError("k={} accepted".format(bad_k))
    for args, exc in (((a, ht.array(np.zeros((4, 2)))), ValueError), ((ht.array(np.zeros((4, 3)), split=1), a),
                                                                      NotImplementedError),
                      ((np.zeros((4, 3)), a), TypeError), ((ht.array(np.zeros((4, 3), dtype=np.int64)), a), None)):
        try:
            ht.spatial.cdist_topk(*args)
        except Exception as e:   # noqa: BLE001 - the exact type is checked below
            assert exc is not None and isinstance(e, exc), (args, e)
        else:
            assert exc is None, args          # integer input promotes to float32 (like cdist)
