"""Deeper parity with ``heat/core/tests/test_statistics.py``: every reduction on UNBALANCED layouts
(skewed lshape maps with empty ranks), every axis incl. tuples and negative axes, keepdims, out=,
integer / bool / float64 inputs, NaN handling, ties in arg-reductions (first index wins), the
moments (mean / var / std / skew / kurtosis) against fp64 NumPy / SciPy-free closed forms, and
the reference's error cases (test_statistics.py assertRaises blocks)."""
import numpy as np

import heat_amd as ht

from ._util import close, raises, rng, same, splits
from .manipulations_deep_checks import _skewed

X3 = rng(21).standard_normal((10, 7, 6)).astype(np.float32)
X2 = rng(22).standard_normal((13, 9)).astype(np.float64)
I2 = rng(23).integers(-20, 20, (12, 5)).astype(np.int64)


def _axes(nd):
    return [None] + list(range(nd)) + [-1] + ([(0, 1), (0, 2), (1, 2)] if nd == 3 else [])


def _skew_ref(x, axis, bias=True):
    m = x.mean(axis=axis, keepdims=True)
    d = x - m
    m2 = (d ** 2).mean(axis=axis)
    m3 = (d ** 3).mean(axis=axis)
    g1 = m3 / m2 ** 1.5
    if bias:
        return g1
    n = x.size if axis is None else x.shape[axis]
    return g1 * np.sqrt(n * (n - 1)) / (n - 2)


def _kurt_ref(x, axis, fisher=True, bias=True):
    m = x.mean(axis=axis, keepdims=True)
    d = x - m
    m2 = (d ** 2).mean(axis=axis)
    m4 = (d ** 4).mean(axis=axis)
    g2 = m4 / m2 ** 2
    if not bias:
        n = x.size if axis is None else x.shape[axis]
        g2 = 3.0 + (n - 1) / ((n - 2) * (n - 3)) * ((n + 1) * g2 - 3 * (n - 1))
    return g2 - 3.0 if fisher else g2


def test_sum_prod_mean_all_axes_unbalanced():
    for s in splits(3):
        x = _skewed(X3, s)
        for ax in _axes(3):
            close(ht.sum(x, axis=ax), X3.sum(axis=ax), rtol=1e-4, atol=1e-4)
            close(ht.mean(x, axis=ax), X3.mean(axis=ax), rtol=1e-4, atol=1e-5)
            if ax is not None:
                close(ht.sum(x, axis=ax, keepdim=True), X3.sum(axis=ax, keepdims=True), rtol=1e-4, atol=1e-4)
    small = (X3[:4, :3, :2] * 0.5 + 1.0).astype(np.float32)
    for s in splits(3):
        close(ht.prod(_skewed(small, s), axis=1), small.prod(axis=1), rtol=1e-5)


def test_var_std_ddof_unbalanced():
    for s in splits(2):
        x = _skewed(X2, s)
        for ax in (None, 0, 1, -1):
            for ddof in (0, 1):
                close(ht.var(x, axis=ax, ddof=ddof), X2.var(axis=ax, ddof=ddof), rtol=1e-10, atol=1e-12)
                close(ht.std(x, axis=ax, ddof=ddof), X2.std(axis=ax, ddof=ddof), rtol=1e-10, atol=1e-12)
    for s in splits(3):
        x = _skewed(X3, s)
        for ax in (None, 0, 2, (0, 1)):
            close(ht.var(x, axis=ax), X3.astype(np.float64).var(axis=ax), rtol=1e-4, atol=1e-5)
    raises(NotImplementedError, ht.var, ht.array(X2), ddof=2)   # reference statistics.py:1693-1698
    raises(ValueError, ht.var, ht.array(X2), ddof=-1)
    raises(TypeError, ht.var, ht.array(X2), ddof="1")
    raises(TypeError, ht.std, ht.array(X2), axis="0")


def test_skew_kurtosis_unbalanced():
    for s in splits(2):
        x = _skewed(X2, s)
        for ax in (None, 0, 1):
            for bias in (True, False):
                close(ht.skew(x, axis=ax, unbiased=not bias), _skew_ref(X2, ax, bias), rtol=1e-8, atol=1e-10)
                for fisher in (True, False):
                    close(ht.kurtosis(x, axis=ax, unbiased=not bias, Fischer=fisher),
                          _kurt_ref(X2, ax, fisher, bias), rtol=1e-8, atol=1e-10)


def test_min_max_unbalanced_keepdims_out():
    for s in splits(3):
        x = _skewed(X3, s)
        for ax in _axes(3):
            same(ht.max(x, axis=ax), X3.max(axis=ax))
            same(ht.min(x, axis=ax), X3.min(axis=ax))
        same(ht.max(x, axis=1, keepdim=True), X3.max(axis=1, keepdims=True))
        same(ht.min(x, axis=(0, 2), keepdim=True), X3.min(axis=(0, 2), keepdims=True))
    for s in splits(2):
        x = _skewed(I2, s)
        same(ht.max(x, axis=0), I2.max(axis=0))
        same(ht.min(x), I2.min())
        out = ht.zeros((5,), dtype=ht.int64)
        ht.max(x, axis=0, out=out)
        same(out, I2.max(axis=0))
    raises(TypeError, ht.max, ht.array(X2), axis="0")
    raises(ValueError, ht.max, ht.array(X2), axis=2)


def test_argmax_argmin_ties_and_nan():
    d = np.array([[1, 5, 5], [5, 2, 0], [5, 5, 1], [0, 0, 0]], dtype=np.float32)
    for s in splits(2):
        x = _skewed(d, s)
        same(ht.argmax(x), np.argmax(d))
        same(ht.argmin(x), np.argmin(d))
        for ax in (0, 1):
            same(ht.argmax(x, axis=ax), np.argmax(d, axis=ax))
            same(ht.argmin(x, axis=ax), np.argmin(d, axis=ax))
        same(ht.argmax(x, axis=1, keepdim=True), np.argmax(d, axis=1)[:, None])
    n = X2.copy()
    n[4, 3] = np.nan
    for s in splits(2):
        x = _skewed(n, s)
        # torch semantics (the reference's backend): NaN is the maximum and the minimum
        same(ht.argmax(x), 4 * 9 + 3)
        same(ht.argmax(x, axis=0)[3], 4)
    for s in splits(2):
        x = _skewed(I2, s)
        same(ht.argmax(x, axis=0), np.argmax(I2, axis=0))
        same(ht.argmin(x), np.argmin(I2))
    out = ht.zeros((9,), dtype=ht.int64)
    ht.argmax(ht.array(X2, split=0), axis=0, out=out)
    same(out, np.argmax(X2, axis=0))
    raises(TypeError, ht.argmax, ht.array(X2), axis="0")
    raises(TypeError, ht.argmin, ht.array(X2), axis=(0, 1))


def test_maximum_minimum_broadcast_splits():
    b = rng(24).standard_normal((1, 9))
    for s in splits(2):
        x = _skewed(X2, s)
        same(ht.maximum(x, ht.array(b)), np.maximum(X2, b))
        same(ht.minimum(x, ht.array(X2[::-1].copy(), split=s)), np.minimum(X2, X2[::-1]))
        same(ht.maximum(x, 0.25), np.maximum(X2, 0.25))
    raises(ValueError, ht.maximum, ht.array(X2), ht.array(np.ones((3, 3))))
    raises(TypeError, ht.minimum, ht.array(X2), "x")


def test_average_weights_unbalanced():
    w1 = rng(25).random(13)
    w2 = rng(26).random((13, 9))
    for s in splits(2):
        x = _skewed(X2, s)
        close(ht.average(x), np.average(X2))
        close(ht.average(x, axis=0, weights=ht.array(w1)), np.average(X2, axis=0, weights=w1), rtol=1e-10)
        close(ht.average(x, axis=1, weights=ht.array(w2, split=s)), np.average(X2, axis=1, weights=w2), rtol=1e-10)
        avg, sw = ht.average(x, axis=0, weights=ht.array(w1), returned=True)
        close(avg, np.average(X2, axis=0, weights=w1), rtol=1e-10)
        close(sw, np.full(9, w1.sum()), rtol=1e-10)
    raises(TypeError, ht.average, ht.array(X2), weights=ht.array(w1))
    raises(ValueError, ht.average, ht.array(X2), axis=0, weights=ht.array(np.ones(5)))
    raises(ZeroDivisionError, ht.average, ht.array(X2), axis=0, weights=ht.zeros(13))


def test_percentile_median_unbalanced():
    for s in splits(2):
        x = _skewed(X2, s)
        for q in (0, 12.5, 50, 99, 100):
            close(ht.percentile(x, q), np.percentile(X2, q), rtol=1e-10)
            for ax in (0, 1):
                close(ht.percentile(x, q, axis=ax), np.percentile(X2, q, axis=ax), rtol=1e-10)
        close(ht.percentile(x, [10, 60], axis=0), np.percentile(X2, [10, 60], axis=0), rtol=1e-10)
        close(ht.median(x, axis=1), np.median(X2, axis=1), rtol=1e-10)
        close(ht.median(x), np.median(X2), rtol=1e-10)
        for method in ("lower", "higher", "nearest", "midpoint"):
            close(ht.percentile(x, 37, axis=0, interpolation=method),
                  np.percentile(X2, 37, axis=0, method=method), rtol=1e-10)
    raises(ValueError, ht.percentile, ht.array(X2), 101)
    raises(ValueError, ht.percentile, ht.array(X2), 50, interpolation="bogus")


def test_cov_variants():
    d = rng(27).standard_normal((4, 30))
    for s in (None, 0, 1):
        x = _skewed(d, s)
        close(ht.cov(x), np.cov(d), rtol=1e-10, atol=1e-12)
        close(ht.cov(x, bias=True), np.cov(d, bias=True), rtol=1e-10, atol=1e-12)
        close(ht.cov(x, ddof=3), np.cov(d, ddof=3), rtol=1e-10, atol=1e-12)
    y = rng(28).standard_normal((2, 30))
    close(ht.cov(ht.array(d, split=1), ht.array(y, split=1)), np.cov(d, y), rtol=1e-10, atol=1e-12)
    close(ht.cov(ht.array(d.T, split=0), rowvar=False), np.cov(d.T, rowvar=False), rtol=1e-10, atol=1e-12)
    raises(TypeError, ht.cov, d)
    raises(ValueError, ht.cov, ht.array(np.ones((2, 2, 2))))
    raises(TypeError, ht.cov, ht.array(d), ddof=1.5)


def test_bincount_histc_unbalanced():
    v = rng(29).integers(0, 7, 40).astype(np.int64)
    w = rng(30).random(40)
    for s in (None, 0):
        x = _skewed(v, s)
        same(ht.bincount(x), np.bincount(v))
        close(ht.bincount(x, weights=ht.array(w, split=s)), np.bincount(v, weights=w), rtol=1e-12)
        same(ht.bincount(x, minlength=12), np.bincount(v, minlength=12))
    f = rng(31).random(50).astype(np.float32) * 10
    for s in (None, 0):
        x = _skewed(f, s)
        h = ht.histc(x, bins=5, min=0, max=10)
        same(h, np.histogram(f, bins=5, range=(0, 10))[0].astype(np.float32))
    raises(ValueError, ht.bincount, ht.array(np.array([[1, 2]], dtype=np.int64)))


def test_reductions_bool_and_empty_rank_layouts():
    b = rng(32).random((9, 4)) > 0.5
    for s in splits(2):
        x = _skewed(b, s)
        same(ht.sum(x, axis=0), b.sum(axis=0))
        same(ht.any(x, axis=1), b.any(axis=1))
        same(ht.all(x, axis=0), b.all(axis=0))
    # a single row: more ranks than rows leaves most ranks empty
    one = X2[:1]
    for s in (None, 0):
        x = ht.array(one, split=s)
        close(ht.mean(x, axis=0), one.mean(axis=0))
        close(ht.var(x, axis=0), one.var(axis=0), atol=1e-12)
        same(ht.argmin(x, axis=0), np.argmin(one, axis=0))
        same(ht.max(x, axis=1), one.max(axis=1))
