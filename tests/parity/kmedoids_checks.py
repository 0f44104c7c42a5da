"""Parity with ``heat/cluster/tests/test_kmedoids.py``: estimator traits, parameters, iris fits
with both initialisations, split-1 and bad-init errors, and recovery of 4 spherical clusters
(float32/float64/int32) - the centres found must lie within one cluster radius of the truth."""
import heat_amd as ht

from ._ml import kcluster_suite

_SUITE = kcluster_suite(ht.cluster.KMedoids, {"n_clusters": 8, "init": "random", "max_iter": 300, "random_state": None})
_REF = "heat/cluster/tests/test_kmedoids.py"


def test_clusterer():
    """KMedoids is a clusterer and not a classifier/regressor (reference ``test_kmedoids.py``)."""
    _SUITE[0]()


def test_get_and_set_params():
    """Default parameters, set_params round trip (reference ``test_kmedoids.py``)."""
    _SUITE[1]()


def test_fit_iris_unsplit():
    """Iris fits with both initialisations, unsplit and split 0: centres of the right shape, labels
    in range, fitted clusters covering the data (reference ``test_kmedoids.py``)."""
    _SUITE[2]()


def test_exceptions():
    """Split-1 input and bad initial centres raise (reference ``test_kmedoids.py``)."""
    _SUITE[3]()


def test_spherical_clusters():
    """Four well-separated spherical clusters (float32 / float64 / int32) are recovered: every
    centre within one cluster radius of the truth (reference ``test_kmedoids.py``)."""
    _SUITE[4]()
