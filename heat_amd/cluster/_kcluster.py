"""
Base of the k-statistics clusterers (reference ``heat/cluster/_kcluster.py``: ``_KCluster`` 10,
``_initialize_cluster_centers`` 87, ``_assign_to_cluster`` 196, ``predict`` 237).

Assignment runs the fused native kernel (``ops.kmeans_assign``: distance GEMM + running argmin,
no n x k matrix) on each rank's block; no communication is needed because the centroids are
replicated. Initialisation draws all k sample positions in ONE Threefry call and fetches the k
rows with ONE distributed take (the reference does k randint calls and k broadcasts).
"""
from __future__ import annotations

from typing import Callable, Optional, Union

import torch

from .. import core as ht
from ..core.base import BaseEstimator, ClusteringMixin
from ..core.communication import MPI
from ..core.dndarray import DNDarray
from .. import ops


class _KCluster(ClusteringMixin, BaseEstimator):
    """Base class for k-means, k-medians and k-medoids."""

    def __init__(self, metric: Callable, n_clusters: int, init: Union[str, DNDarray], max_iter: int, tol: float,
                 random_state: Optional[int]):
        self.n_clusters = n_clusters
        self.init = init
        self.max_iter = max_iter
        self.tol = tol
        self.random_state = random_state
        self._metric = metric
        self._cluster_centers = None
        self._labels = None
        self._inertia = None
        self._n_iter = None
        # "fast": fp16x3 split assignment (fp32-GEMM accuracy, points packed once per fit);
        # "exact": bit-exact fp32 (f32-input MFMA) assignment
        self.precision = "fast"
        self._pack_cache = None
        # certified one-term assignment (ops.kmeans_assign(certified=True)) while it pays: every
        # certified call posts its re-check count to the host (pinned copy + event); the next call
        # waits for that event (the previous iteration, normally finished) and decides. Once more
        # than CERT_MAX_RECHECK of the points needed the 3-term re-run (the filter costs ~55 % of
        # the full kernel, the re-run of a fraction q about q of it), the full kernel takes over
        # until the points change.
        self._certify = True
        self._cert_probe = None
        self._cert_calls = 0

    CERT_MAX_RECHECK = 0.35

    def _assign_labels(self, X: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
        """int32 nearest-centroid labels of the local points (native fused kernels)."""
        # the fp16x3 planes serve the MFMA kernels only (k <= 16 runs the exact VALU kernel)
        packed = self._packed(X) if X.dtype == torch.float32 and not ops.kernels._small_k_ok(X, C.shape[0]) \
            else None
        probe = self._cert_probe
        if probe is not None:
            # an asynchronous fit loop runs ahead of the GPU: waiting here (for the previous
            # iteration) is what makes the decision happen at all
            probe[1].synchronize()
            self._certify = probe[0].item() <= self.CERT_MAX_RECHECK * probe[2]
            self._cert_probe = probe = None
        certified = packed is not None and self._certify
        labels, _ = ops.kmeans_assign(X, C, want_mind=False, packed=packed, certified=certified)
        self._cert_calls += 1
        if certified and X.shape[0] > 0:
            host = torch.empty(1, dtype=torch.int32, pin_memory=True)
            host.copy_(ops.kernels.kmeans_assign.last_rechecked.reshape(1), non_blocking=True)  # unwrapped by profiling
            ev = torch.cuda.Event()
            ev.record()
            self._cert_probe = (host, ev, X.shape[0])
        return labels

    def _packed(self, X: torch.Tensor):
        """fp16x3 planes of the local points, cached while X is unchanged (None: exact path)."""
        if self.precision != "fast" or not X.is_cuda:
            return None
        key = ops.kernels._points_key(X)
        if self._pack_cache is None or self._pack_cache.key != key:
            self._pack_cache = None
            self._certify, self._cert_probe, self._cert_calls = True, None, 0
            self._pack_cache = ops.kmeans_pack_points(X)
        return self._pack_cache

    @property
    def cluster_centers_(self) -> DNDarray:
        # handed out: the caller may write into it by any path, so the next step re-pads it
        self._own_newC = None
        return self._cluster_centers

    @property
    def labels_(self) -> DNDarray:
        return self._labels

    @property
    def inertia_(self) -> float:
        # step() with tol=None keeps the shift as a device scalar (no host sync per step); the
        # property hands out the float the reference returns
        if self._inertia is not None and not isinstance(self._inertia, float):
            self._inertia = float(self._inertia)
        return self._inertia

    @property
    def n_iter_(self) -> int:
        return self._n_iter

    # ------------------------------------------------------------------------------ helpers
    @staticmethod
    def _rows(x: DNDarray, idx: torch.Tensor) -> torch.Tensor:
        """Replicated copy of the rows ``idx`` (global indices) of a split-0 / replicated array."""
        if not x.is_distributed():
            return x.larray[idx.to(x.larray.device)]
        return x[idx]._gathered()

    def _initialize_cluster_centers(self, x: DNDarray):
        if self.random_state is not None:
            ht.random.seed(self.random_state)
        k = self.n_clusters
        n, f = x.gshape
        if isinstance(self.init, DNDarray):
            if self.init.ndim != 2:
                raise ValueError("passed centroids need to be two-dimensional, but are {}".format(self.init.ndim))
            if self.init.gshape[0] != k or self.init.gshape[1] != f:
                raise ValueError("passed centroids do not match cluster count or data shape")
            c = self.init._gathered() if self.init.is_distributed() else self.init.larray
            self._cluster_centers = DNDarray(c.to(x.larray.dtype).to(x.larray.device).clone(), (k, f), x.dtype, None,
                                             x.device, x.comm, True)
            return
        if x.split not in (None, 0):
            raise NotImplementedError("Not implemented for other splitting-axes")
        if self.init == "random":
            # one sample per stratum [n//k*i, n//k*(i+1)) like the reference, drawn in one call
            u = ht.random.rand(k, dtype=ht.float64, device="cpu").larray
            width = n // k
            lo = torch.arange(k, dtype=torch.float64) * width
            idx = (lo + torch.floor(u * max(width, 1))).to(torch.int64).clamp(max=n - 1)
            c = self._rows(x, idx)
        elif self.init in ("probability_based", "kmeans++"):
            c = self._kmeanspp(x)
        else:
            raise ValueError('init needs to be one of "random", ht.DNDarray or "kmeans++", but was {}'.format(self.init))
        self._cluster_centers = DNDarray(c.contiguous(), (k, f), x.dtype, None, x.device, x.comm, True)

    def _kmeanspp(self, x: DNDarray) -> torch.Tensor:
        """k-means++ seeding with an incrementally maintained D^2 (O(n f) per new centroid)."""
        k = self.n_clusters
        n, f = x.gshape
        X = x.larray
        first = int(ht.random.randint(0, n, size=(1,), device="cpu").larray.item())
        cents = [self._rows(x, torch.tensor([first]))[0]]
        d2 = ((X - cents[0]) ** 2).sum(1)
        counts, displs = (x.counts_displs() if x.is_distributed() else ((n,), (0,)))
        me = x.comm.rank if x.is_distributed() else 0
        for _ in range(1, k):
            local = d2.sum().reshape(1).double()
            sums = x.comm.allgather_tensor(local, 0).cpu() if x.is_distributed() else local.cpu()
            total = float(sums.sum())
            r = float(ht.random.rand(1, dtype=ht.float64, device="cpu").larray.item()) * total
            # owner rank: first whose cumulative sum exceeds r
            cum = torch.cumsum(sums, 0)
            owner = int(torch.searchsorted(cum, torch.tensor([r], dtype=cum.dtype), right=True).clamp(max=len(cum) - 1))
            if me == owner:
                rr = r - (float(cum[owner - 1]) if owner > 0 else 0.0)
                lc = torch.cumsum(d2.double(), 0)
                li = int(torch.searchsorted(lc, torch.tensor([rr], dtype=lc.dtype, device=lc.device), right=True)
                         .clamp(max=max(len(lc) - 1, 0)))
                row = X[li].clone()
            else:
                row = torch.empty(f, dtype=X.dtype, device=X.device)
            if x.is_distributed():
                x.comm.Bcast(row, root=owner)
            cents.append(row)
            d2 = torch.minimum(d2, ((X - row) ** 2).sum(1))
        return torch.stack(cents)

    def _assign_to_cluster(self, x: DNDarray) -> DNDarray:
        """(n, 1) int64 labels of the nearest centroid (split like ``x``)."""
        X = x.larray
        labels = self._assign_labels(X, self._cluster_centers.larray.to(X.device))
        lab = labels.to(torch.int64).reshape(-1, 1)
        return DNDarray(lab, (x.gshape[0], 1), ht.int64, x.split, x.device, x.comm, x.balanced)

    def _update_centroids(self, x: DNDarray, matching_centroids: DNDarray):
        raise NotImplementedError()

    def fit(self, x: DNDarray):
        raise NotImplementedError()

    def predict(self, x: DNDarray) -> DNDarray:
        """Index of the closest centroid for every sample (shape (n, 1))."""
        if not isinstance(x, DNDarray):
            raise ValueError("input needs to be a ht.DNDarray, but was {}".format(type(x)))
        if x.split is not None and x.split != 0:
            raise NotImplementedError("Not implemented for other splitting-axes")
        return self._assign_to_cluster(x)


# ---------------------------------------------------------------------------------------------
# exact per-cluster order statistics (medians) without sorting or gathering the data
# ---------------------------------------------------------------------------------------------
def _ordered_keys(X: torch.Tensor) -> torch.Tensor:
    """Monotone map float -> int64 (bit-level): x < y  <=>  key(x) < key(y)."""
    if X.dtype == torch.float64:
        i = X.view(torch.int64)
        return i ^ ((i >> 63) & 0x7FFFFFFFFFFFFFFF)
    i = X.float().view(torch.int32).to(torch.int64)
    return i ^ ((i >> 31) & 0x7FFFFFFF)


def _keys_to_values(K: torch.Tensor, dtype) -> torch.Tensor:
    if dtype == torch.float64:
        return (K ^ ((K >> 63) & 0x7FFFFFFFFFFFFFFF)).view(torch.float64)
    k32 = (K ^ ((K >> 31) & 0x7FFFFFFF)).to(torch.int32)
    return k32.view(torch.float32)


def cluster_medians(X: torch.Tensor, labels: torch.Tensor, k: int, comm, distributed: bool):
    """Exact per-(cluster, feature) medians of the rows of X grouped by ``labels``.

    Bisection on the bit-ordered integer keys: every step counts, per (cluster, feature), the
    members below the probe with one pass and ONE all-reduce of 2*k*f counts; <= 64 steps give
    the exact lower/upper middle order statistics (averaged like NumPy's median).
    Returns (medians [k, f], counts [k])."""
    n, f = X.shape
    lab = labels.reshape(-1).to(torch.int64)
    dev = X.device
    cnt = torch.bincount(lab, minlength=k).to(torch.float64)
    keys = _ordered_keys(X)
    if n:
        kmin = keys.min(0).values
        kmax = keys.max(0).values
    else:
        big = (1 << 62)
        kmin = torch.full((f,), big, dtype=torch.int64, device=dev)
        kmax = torch.full((f,), -big, dtype=torch.int64, device=dev)
    if distributed:
        comm.Allreduce(MPI.IN_PLACE, cnt, MPI.SUM)
        comm.Allreduce(MPI.IN_PLACE, kmin, MPI.MIN)
        comm.Allreduce(MPI.IN_PLACE, kmax, MPI.MAX)
    c = cnt.to(torch.int64)
    t = torch.stack([(c - 1).clamp(min=0) // 2, c // 2])                  # [2, k] target ranks
    lo = kmin.unsqueeze(0).unsqueeze(0).expand(2, k, f).clone()
    hi = kmax.unsqueeze(0).unsqueeze(0).expand(2, k, f).clone()
    need = (t + 1).unsqueeze(-1).to(torch.float64)                       # [2, k, 1]
    for _ in range(70):
        if bool((lo >= hi).all()):
            break
        mid = (lo >> 1) + (hi >> 1) + (lo & hi & 1)  # floor((lo+hi)/2) without overflow
        counts = torch.zeros((2, k, f), dtype=torch.float64, device=dev)
        for s in range(2):
            le = (keys <= mid[s][lab]).to(torch.float64)                  # [n, f]
            counts[s].index_add_(0, lab, le)
        if distributed:
            comm.Allreduce(MPI.IN_PLACE, counts, MPI.SUM)
        ok = counts >= need
        hi = torch.where(ok, mid, hi)
        lo = torch.where(ok, lo, mid + 1)
    vals = _keys_to_values(lo, X.dtype if X.dtype == torch.float64 else torch.float32)
    med = ((vals[0].double() + vals[1].double()) / 2).to(X.dtype)
    return med, cnt
