"""
K-Medoids (reference ``heat/cluster/kmedoids.py``: ``_update_centroids`` 60-121, ``fit`` 123).

The medoid of each cluster is the member closest to the cluster's median; all clusters are
handled at once: medians by bisection (``cluster_medians``), the closest member per cluster by a
segmented min + ONE all-reduce of k minima and ONE of k first indices.
"""
from __future__ import annotations

from typing import Optional, Union

import torch

from .. import core as ht
from ..core.communication import MPI
from ..core.dndarray import DNDarray
from ._kcluster import _KCluster, cluster_medians


class KMedoids(_KCluster):
    """K-Medoids clustering: centroids are always data points."""

    def __init__(self, n_clusters: int = 8, init: Union[str, DNDarray] = "random", max_iter: int = 300,
                 random_state: Optional[int] = None):
        if isinstance(init, str) and init == "kmedoids++":
            init = "probability_based"
        super().__init__(metric=lambda x, y: ht.spatial.distance.manhattan(x, y, expand=True), n_clusters=n_clusters,
                         init=init, max_iter=max_iter, tol=0.0, random_state=random_state)

    def _assign_to_cluster(self, x: DNDarray) -> DNDarray:
        from .. import ops

        d = ops.cdist(x.larray.float() if not x.larray.is_floating_point() else x.larray,
                      self._cluster_centers.larray.to(x.larray.device), "manhattan")
        lab = torch.argmin(d, dim=1).to(torch.int64).reshape(-1, 1)
        return DNDarray(lab, (x.gshape[0], 1), ht.int64, x.split, x.device, x.comm, x.balanced)

    def _update_centroids(self, x: DNDarray, matching_centroids: DNDarray) -> DNDarray:
        k = self.n_clusters
        X = x.larray if x.larray.is_floating_point() else x.larray.float()
        lab = matching_centroids.larray.reshape(-1).to(torch.int64)
        dist = x.is_distributed()
        med, cnt = cluster_medians(X, lab, k, x.comm, dist)
        d = (X - med[lab]).abs().sum(1).double() if X.shape[0] else X.new_zeros(0, dtype=torch.float64)
        inf = float("inf")
        best = torch.full((k,), inf, dtype=torch.float64, device=X.device)
        if X.shape[0]:
            best.scatter_reduce_(0, lab, d, reduce="amin")
        if dist:
            x.comm.Allreduce(MPI.IN_PLACE, best, MPI.MIN)
        off = x.counts_displs()[1][x.comm.rank] if dist else 0
        gidx = torch.arange(X.shape[0], device=X.device, dtype=torch.int64) + off
        big = torch.iinfo(torch.int64).max
        first = torch.full((k,), big, dtype=torch.int64, device=X.device)
        if X.shape[0]:
            hit = d == best[lab]
            first.scatter_reduce_(0, lab[hit], gidx[hit], reduce="amin")
        if dist:
            x.comm.Allreduce(MPI.IN_PLACE, first, MPI.MIN)
        C = self._cluster_centers.larray
        valid = first != big
        newC = C.clone()
        if bool(valid.any()):
            rows = self._rows(x, first[valid].cpu())
            newC[valid.to(C.device)] = rows.to(C.dtype).to(C.device)
        return DNDarray(newC, C.shape, self._cluster_centers.dtype, None, x.device, x.comm, True)

    def fit(self, x: DNDarray) -> "KMedoids":
        if not isinstance(x, DNDarray):
            raise ValueError("input needs to be a ht.DNDarray, but was {}".format(type(x)))
        self._initialize_cluster_centers(x)
        self._n_iter = 0
        matching = None
        for _ in range(self.max_iter):
            self._n_iter += 1
            matching = self._assign_to_cluster(x)
            new = self._update_centroids(x, matching)
            if torch.equal(self._cluster_centers.larray, new.larray):
                break
            self._cluster_centers = new
        self._labels = matching
        return self
