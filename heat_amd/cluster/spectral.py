"""
Spectral clustering (reference ``heat/cluster/spectral.py``: ``Spectral`` 12, ``_spectral_embedding``
103, ``fit`` 134, ``predict`` 175): Laplacian -> Lanczos (batched re-orthogonalisation) ->
eigen-decomposition of the small tridiagonal T -> KMeans on the first k eigenvectors.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch

from .. import core as ht
from ..core.base import BaseEstimator, ClusteringMixin
from ..core.dndarray import DNDarray
from .kmeans import KMeans
from .. import graph, spatial


class Spectral(ClusteringMixin, BaseEstimator):
    """Spectral clustering with an RBF or euclidean similarity graph."""

    def __init__(self, n_clusters: int = None, gamma: float = 1.0, metric: str = "rbf",
                 laplacian: str = "fully_connected", threshold: float = 1.0, boundary: str = "upper",
                 n_lanczos: int = 300, assign_labels: str = "kmeans", **params):
        self.n_clusters = n_clusters
        self.gamma = gamma
        self.metric = metric
        self.laplacian = laplacian
        self.threshold = threshold
        self.boundary = boundary
        self.n_lanczos = n_lanczos
        self.assign_labels = assign_labels
        if metric == "rbf":
            sig = math.sqrt(1 / (2 * gamma))
            self._laplacian = graph.Laplacian(lambda x: spatial.rbf(x, sigma=sig, quadratic_expansion=True),
                                                 definition="norm_sym", mode=laplacian, threshold_key=boundary,
                                                 threshold_value=threshold)
        elif metric == "euclidean":
            self._laplacian = graph.Laplacian(lambda x: spatial.cdist(x, quadratic_expansion=True),
                                                 definition="norm_sym", mode=laplacian, threshold_key=boundary,
                                                 threshold_value=threshold)
        else:
            raise NotImplementedError("Other kernels currently not supported")
        if assign_labels == "kmeans":
            # options for the label-assigning k-means, flat or as params={...}; keys k-means does not
            # take (e.g. the reference's normalize=) are accepted and ignored, like the reference
            opts = dict(params.pop("params", None) or {})
            opts.update(params)
            known = ("init", "max_iter", "tol", "random_state")
            self._cluster = KMeans(**{k: v for k, v in opts.items() if k in known})
        else:
            raise NotImplementedError("Other Label Assignment Algorithms are currently not available")
        self._labels = None
        self._cluster_centers = None

    @property
    def labels_(self) -> DNDarray:
        return self._labels

    def _spectral_embedding(self, x: DNDarray) -> Tuple[DNDarray, DNDarray]:
        L = self._laplacian.construct(x)
        n = L.gshape[0]
        m = min(self.n_lanczos, n)
        v0 = ht.full((n,), fill_value=1.0 / math.sqrt(n), dtype=L.dtype, split=0 if L.split is not None else None,
                     device=L.device, comm=L.comm)
        V, T = ht.lanczos(L, m, v0)
        evals, evecs = torch.linalg.eigh(T.larray.double())
        evals, idx = torch.sort(evals)
        evecs = evecs[:, idx].to(T.larray.dtype)
        eigenvalues = ht.array(evals.to(T.larray.dtype), device=L.device, comm=L.comm)
        # V stays row-split: every rank forms its own rows of V @ evecs (n x m basis never gathered)
        vec = V.larray @ evecs.to(V.larray.dtype)
        if V.split == 0:
            eigenvectors = ht.DNDarray(vec, (n, vec.shape[1]), ht.types.canonical_heat_type(vec.dtype), 0, L.device,
                                       L.comm, V.balanced)
        else:
            eigenvectors = ht.array(vec, split=0 if x.split == 0 else None, device=L.device, comm=L.comm)
        return eigenvalues, eigenvectors

    def fit(self, x: DNDarray) -> "Spectral":
        if not isinstance(x, DNDarray):
            raise ValueError("input needs to be a ht.DNDarray, but was {}".format(type(x)))
        if x.split is not None and x.split != 0:
            raise NotImplementedError("Not implemented for other splitting-axes")
        eigenvalues, eigenvectors = self._spectral_embedding(x)
        if self.n_clusters is None:
            ev = eigenvalues.larray
            diff = ev[1:] - ev[:-1]
            self.n_clusters = int(torch.argmax(diff).item()) + 1
        components = eigenvectors[:, : self.n_clusters].copy()
        params = self._cluster.get_params()
        params["n_clusters"] = self.n_clusters
        self._cluster.set_params(**params)
        self._cluster.fit(components)
        self._labels = self._cluster.labels_
        self._cluster_centers = self._cluster.cluster_centers_
        return self

    def predict(self, x: DNDarray) -> DNDarray:
        if not isinstance(x, DNDarray):
            raise ValueError("input needs to be a ht.DNDarray, but was {}".format(type(x)))
        if x.split is not None and x.split != 0:
            raise NotImplementedError("Not implemented for other splitting-axes")
        _, eigenvectors = self._spectral_embedding(x)
        components = eigenvectors[:, : self.n_clusters].copy()
        return self._cluster.predict(components)
