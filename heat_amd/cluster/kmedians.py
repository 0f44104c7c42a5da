"""
K-Medians (reference ``heat/cluster/kmedians.py``: ``_update_centroids`` 60-110, ``fit`` 112).

The per-cluster medians of all clusters and features are found together by bisection on the
bit-ordered keys (``cluster_medians``: one pass + one all-reduce of 2*k*f counts per step), instead
of the reference's k distributed sorts per iteration.
"""
from __future__ import annotations

from typing import Optional, Union

import torch

from .. import core as ht
from ..core.dndarray import DNDarray
from ._kcluster import _KCluster, cluster_medians


class KMedians(_KCluster):
    """K-Medians clustering (Manhattan assignment metric, median update)."""

    def __init__(self, n_clusters: int = 8, init: Union[str, DNDarray] = "random", max_iter: int = 300,
                 tol: float = 1e-4, random_state: Optional[int] = None):
        if isinstance(init, str) and init == "kmedians++":
            init = "probability_based"
        super().__init__(metric=lambda x, y: ht.spatial.distance.manhattan(x, y, expand=True), n_clusters=n_clusters,
                         init=init, max_iter=max_iter, tol=tol, random_state=random_state)

    def _assign_to_cluster(self, x: DNDarray) -> DNDarray:
        from .. import ops

        d = ops.cdist(x.larray.float() if not x.larray.is_floating_point() else x.larray,
                      self._cluster_centers.larray.to(x.larray.device), "manhattan")
        lab = torch.argmin(d, dim=1).to(torch.int64).reshape(-1, 1)
        return DNDarray(lab, (x.gshape[0], 1), ht.int64, x.split, x.device, x.comm, x.balanced)

    def _update_centroids(self, x: DNDarray, matching_centroids: DNDarray) -> DNDarray:
        X = x.larray if x.larray.is_floating_point() else x.larray.float()
        med, cnt = cluster_medians(X, matching_centroids.larray, self.n_clusters, x.comm, x.is_distributed())
        C = self._cluster_centers.larray
        newC = torch.where(cnt.unsqueeze(1) > 0, med.to(C.dtype), C)
        return DNDarray(newC, C.shape, self._cluster_centers.dtype, None, x.device, x.comm, True)

    def fit(self, x: DNDarray) -> "KMedians":
        if not isinstance(x, DNDarray):
            raise ValueError("input needs to be a ht.DNDarray, but was {}".format(type(x)))
        self._initialize_cluster_centers(x)
        self._n_iter = 0
        matching = None
        for _ in range(self.max_iter):
            self._n_iter += 1
            matching = self._assign_to_cluster(x)
            new = self._update_centroids(x, matching)
            self._inertia = float(((self._cluster_centers.larray - new.larray) ** 2).sum())
            self._cluster_centers = new
            if self.tol is not None and self._inertia <= self.tol:
                break
        self._labels = matching
        return self
