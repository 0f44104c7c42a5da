"""Shared fixtures for the estimator parity checks."""
from __future__ import annotations

import os

import numpy as np

import heat_amd as ht

DS = "/root/reference/heat/datasets"


def iris(split=None):
    """The reference's iris table (``iris.csv``, a plain data file) or a synthetic stand-in."""
    p = os.path.join(DS, "iris.csv")
    if os.path.exists(p):
        return ht.load(p, sep=";", split=split)
    from heat_amd.datasets import iris as synth

    return synth(split=split)[0]


def iris_labels():
    return np.repeat(np.arange(3), 50)


def spherical(n_per_cluster, radius=1.0, offset=4.0, dtype=ht.float32, seed=1, split=0):
    """4 ball-shaped clusters in 3-D centred at (o,o,o), (2o,2o,2o), (-o,-o,-o), (2o,-2o,-2o) - the
    reference's ``create_spherical_dataset`` layout - plus the true centres."""
    rng = np.random.default_rng(seed)
    centres = np.array([[offset] * 3, [2 * offset] * 3, [-offset] * 3, [2 * offset, -2 * offset, -2 * offset]])
    pts = []
    for c in centres:
        r = rng.random(n_per_cluster) * radius
        th = rng.random(n_per_cluster) * np.pi
        ph = rng.random(n_per_cluster) * 2 * np.pi
        pts.append(np.stack([r * np.sin(th) * np.cos(ph), r * np.sin(th) * np.sin(ph), r * np.cos(th)], 1) + c)
    x = np.concatenate(pts)
    npdt = {ht.float32: np.float32, ht.float64: np.float64, ht.int32: np.int32}[dtype]
    return ht.array(x.astype(npdt), split=split), centres


def kcluster_suite(cls, defaults):
    """clusterer / params / iris / exceptions / spherical checks shared by KMeans, KMedians, KMedoids."""
    def test_clusterer():
        c = cls()
        assert ht.is_estimator(c) and ht.is_clusterer(c)

    def test_get_and_set_params():
        c = cls()
        params = c.get_params()
        assert params == defaults, params
        params["n_clusters"] = 10
        c.set_params(**params)
        assert c.n_clusters == 10

    def test_fit_iris_unsplit():
        for split in (None, 0):
            x = iris(split)
            for init in ("random", "kmeans++" if cls is not ht.cluster.KMedoids else "kmedoids++"):
                c = cls(n_clusters=3, init=init, random_state=1)
                c.fit(x)
                assert isinstance(c.cluster_centers_, ht.DNDarray) and c.cluster_centers_.shape == (3, 4)
                lab = c.predict(x)
                assert lab.shape[0] == 150
                # clusters are consistent with the (well separated) setosa class
                v = lab.numpy().reshape(-1)
                assert len(set(v[:50].tolist())) == 1 and v[0] not in set(v[50:].tolist())

    def test_exceptions():
        x = iris(1)
        c = cls(n_clusters=3)
        try:
            c.fit(x)
            raise AssertionError("fit of split=1 data did not raise")
        except NotImplementedError:
            pass
        try:
            c.set_params(foo="bar")
            raise AssertionError("set_params(foo=...) did not raise")
        except ValueError:
            pass
        try:
            cls(n_clusters=3, init="random_number").fit(iris(0))
            raise AssertionError("bad init did not raise")
        except ValueError:
            pass

    def test_spherical_clusters():
        p = ht.MPI_WORLD.size
        for n, dtype, radius, offset in ((20 * p, ht.float32, 1.0, 4.0), (100 * p, ht.float32, 1.0, 4.0),
                                         (20 * p, ht.float64, 1.0, 4.0), (20 * p, ht.int32, 10.0, 40.0)):
            x, centres = spherical(n, radius, offset, dtype)
            init = "kmeans++" if cls is not ht.cluster.KMedoids else "kmedoids++"
            c = cls(n_clusters=4, init=init, random_state=3)
            c.fit(x)
            cc = c.cluster_centers_
            assert isinstance(cc, ht.DNDarray) and cc.shape == (4, 3)
            got = np.sort(cc.numpy().astype(np.float64), axis=0)
            want = np.sort(centres, axis=0)
            assert np.abs(got - want).max() < radius * 1.01 + 1e-6, (got, want)

    return test_clusterer, test_get_and_set_params, test_fit_iris_unsplit, test_exceptions, test_spherical_clusters
