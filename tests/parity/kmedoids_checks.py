"""Parity with ``heat/cluster/tests/test_kmedoids.py``: estimator traits, parameters, iris fits
with both initialisations, split-1 and bad-init errors, and recovery of 4 spherical clusters
(float32/float64/int32) - the centres found must lie within one cluster radius of the truth."""
import heat_amd as ht

from ._ml import kcluster_suite

(test_clusterer, test_get_and_set_params, test_fit_iris_unsplit, test_exceptions,
 test_spherical_clusters) = kcluster_suite(ht.cluster.KMedoids, {"n_clusters": 8, "init": "random", "max_iter": 300, "random_state": None})
