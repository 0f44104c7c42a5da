"""
K-Means (Lloyd's algorithm) (reference ``heat/cluster/kmeans.py``: ``KMeans`` 13,
``_update_centroids`` 73-100, ``fit`` 102-139).

Per iteration and rank: ONE fused assign kernel (distances as a 3-term fp16 split on the FP16
matrix cores, ~fp32-GEMM accuracy, plus a running argmax of the score; the points' fp16 planes are
packed once per fit - ``ops/csrc/kmeans_f16x3.hip``; a certified one-term filter with a 3-term
re-check where it pays; k <= 16 a single fused VALU/MFMA pass, ``kmeans_smallk.hip``; the exact
f32-MFMA kernel under ``precision="exact"``), ONE deterministic update (counting sort of the
labels, fixed-order per-cluster sums and counts - ``kmeans.hip``: no float atomics, bit-reproducible
runs) and ONE all-reduce of the packed (k*f sums + k counts) over RCCL - instead of the reference's
k full passes over the data and 2k all-reduces + k broadcasts.
"""
from __future__ import annotations

from typing import Optional, Union

import torch

from .. import core as ht
from ..core.communication import MPI
from ..core.dndarray import DNDarray
from .. import ops
from ._kcluster import _KCluster


class KMeans(_KCluster):
    """K-Means clustering.

    Parameters: ``n_clusters``, ``init`` ('random', 'kmeans++'/'probability_based' or a DNDarray of
    initial centers), ``max_iter``, ``tol`` (convergence on the squared centroid shift, like the
    reference's ``inertia_``), ``random_state``.
    """

    def __init__(self, n_clusters: int = 8, init: Union[str, DNDarray] = "random", max_iter: int = 300,
                 tol: float = 1e-4, random_state: Optional[int] = None):
        if isinstance(init, str) and init == "kmeans++":
            init = "probability_based"
        super().__init__(metric=lambda x, y: ht.spatial.distance.cdist(x, y, quadratic_expansion=True),
                         n_clusters=n_clusters, init=init, max_iter=max_iter, tol=tol, random_state=random_state)

    def _centroid_step(self, X: torch.Tensor, C: torch.Tensor, comm, distributed: bool):
        """One Lloyd step on the local block: returns (new centroids, int32 labels)."""
        k = C.shape[0]
        if not distributed:
            # one process: the whole step is the pass over the points + one epilogue launch
            # the padded centroids of the previous step are reused only for this loop's own output
            step = ops.kmeans_lloyd_small(X, C, reuse_pad=C is getattr(self, "_own_newC", None))
            if step is not None:
                labels, newC, self._step_shift = step
                self._own_newC = newC
                return newC, labels
        fused = ops.kmeans_step_small(X, C)   # exact fp32: serves both precisions
        if fused is not None:   # few clusters: assignment and sums in one pass over the points
            labels, sums, counts = fused
        else:
            labels = self._assign_labels(X, C)
            sums, counts = ops.kmeans_update(X, labels, k)
        if distributed:
            kf = sums.numel()
            packed = torch.empty(kf + k, dtype=torch.float64, device=sums.device)
            packed[:kf].copy_(sums.reshape(-1))
            packed[kf:].copy_(counts)
            comm.Allreduce(MPI.IN_PLACE, packed, MPI.SUM)
            # new centroids + squared shift in one launch (csrc/kmeans_finalize.hip)
            newC, self._step_shift = ops.kmeans_finalize(packed, C)
        else:   # no pack: the epilogue reads the update kernel's fp32 sums and counts directly
            newC, self._step_shift = ops.kmeans_finalize(None, C, sums=sums, counts=counts)
        return newC, labels

    def _update_centroids(self, x: DNDarray, matching_centroids: DNDarray) -> DNDarray:
        """Mean of the points assigned to each centroid (empty clusters keep their centroid)."""
        k = self.n_clusters
        labels = matching_centroids.larray.reshape(-1).to(torch.int32)
        X = x.larray
        sums, counts = ops.kmeans_update(X if X.dtype == torch.float32 else X.float(), labels, k)
        packed = torch.cat([sums.reshape(-1).double(), counts.double()])
        if x.is_distributed():
            x.comm.Allreduce(MPI.IN_PLACE, packed, MPI.SUM)
        gs = packed[: sums.numel()].reshape(sums.shape)
        gc = packed[sums.numel():]
        C = self._cluster_centers.larray
        newC = torch.where(gc.unsqueeze(1) > 0, gs / gc.clamp(min=1).unsqueeze(1), C.double()).to(C.dtype)
        return DNDarray(newC, C.shape, self._cluster_centers.dtype, None, x.device, x.comm, True)

    def _graph_ok(self, X: torch.Tensor, comm, distributed: bool) -> bool:
        """HIP-graph replay of the Lloyd step (``HEAT_KMEANS_GRAPH=1``): device data, no
        certified-assignment probe in flight (it posts to the host), and collectives that are
        stream-ordered on the capturing stream (a world of one, or the native communicator)."""
        import os

        if os.environ.get("HEAT_KMEANS_GRAPH", "0") != "1" or not X.is_cuda:
            return False
        # Measured on MI355X / ROCm 7 (tools/microbench/graph_debug2.py): with the runtime's graph
        # packet capture (the default), replays of a step containing a 256 KB memset node went wrong
        # from the second replay (centroids diverged to 1e27); with
        # DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 they were exact. The update kernels no longer memset
        # (profiles/kmeans_graph_replay_r02.md), but graph mode stays restricted to processes
        # started with that variable (read at HIP init): it is correct there and not faster.
        if os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") != "0":
            return False
        if self._certify or self._cert_probe is not None:
            return False
        if self.precision == "fast" and (self._pack_cache is None or self._pack_cache.key != ops.kernels._points_key(X)):
            return False  # the fp16x3 planes are (re)built eagerly, outside any capture
        if not distributed:
            return True
        # a captured IPC all-reduce would freeze its host-side epoch and slot parity into the graph:
        # every replay would pass its barriers on flags of earlier replays (wrong sums)
        from ..parallel import ipc

        return not ipc.enabled() and comm._native() is not None

    def _centroid_step_graph(self, X: torch.Tensor, C: torch.Tensor, comm, distributed: bool):
        """The Lloyd step replayed from a captured HIP graph: ONE launch per iteration instead of
        ~15 kernel launches and their host overhead. Re-captured when the points, their planes
        or the shapes change."""
        key = (X.data_ptr(), tuple(X.shape), tuple(C.shape), C.dtype, self.precision, distributed,
               id(self._pack_cache))
        g = getattr(self, "_graph", None)
        if g is None or self._graph_key != key:
            self._graph = None
            c_in = C.clone()
            side = torch.cuda.Stream(device=X.device)
            side.wait_stream(torch.cuda.current_stream(X.device))
            with torch.cuda.stream(side):
                self._centroid_step(X, c_in, comm, distributed)  # warm the allocator on this stream
            torch.cuda.current_stream(X.device).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                c_out, labels = self._centroid_step(X, c_in, comm, distributed)
            self._graph, self._graph_key = g, key
            self._graph_io = (c_in, c_out, labels, self._step_shift)
        c_in, c_out, labels, shift = self._graph_io
        c_in.copy_(C)
        g.replay()
        self._step_shift = shift.clone()
        # the graph's buffers are overwritten by the next replay: hand out copies
        return c_out.clone(), labels.clone()

    def step(self, x: DNDarray) -> Union[float, torch.Tensor]:
        """One Lloyd iteration on the current centers (initialising them on first use); returns
        the squared centroid shift (a float, or a 0-d device tensor when ``tol`` is None). The
        building block of :meth:`fit`, exposed for streaming use and benchmarking."""
        if self._cluster_centers is None:
            self._initialize_cluster_centers(x)
            self._n_iter = 0
        X = x.larray if x.larray.is_floating_point() else x.larray.float()
        C = self._cluster_centers.larray.to(X.dtype)
        if self._graph_ok(X, x.comm, x.is_distributed()):
            newC, labels = self._centroid_step_graph(X, C, x.comm, x.is_distributed())
        else:
            newC, labels = self._centroid_step(X, C, x.comm, x.is_distributed())
        shift = self._step_shift
        if self.tol is not None:
            shift = float(shift)  # a convergence test needs the value on the host
        # tol=None (fixed iteration count): the shift stays a device scalar, no host sync per step,
        # so the next step's kernels queue while this one runs (like fit())
        self._cluster_centers = DNDarray(newC, newC.shape, self._cluster_centers.dtype, None, x.device, x.comm, True)
        self._inertia = shift
        self._n_iter = (self._n_iter or 0) + 1
        self._last_labels = labels
        return shift

    def fit(self, x: DNDarray) -> "KMeans":
        """Lloyd iterations until the squared centroid shift is <= ``tol`` or ``max_iter``."""
        if not isinstance(x, DNDarray):
            raise ValueError("input needs to be a ht.DNDarray, but was {}".format(type(x)))
        if x.split is not None and x.split != 0:
            raise NotImplementedError("Not implemented for other splitting-axes")
        self._initialize_cluster_centers(x)
        X = x.larray
        if not X.is_floating_point():
            X = X.float()
        C = self._cluster_centers.larray.to(X.dtype)
        distributed = x.is_distributed()
        labels = None
        self._n_iter = 0
        for _ in range(self.max_iter):
            self._n_iter += 1
            newC, labels = self._centroid_step(X, C, x.comm, distributed)
            shift = self._step_shift
            C = newC
            if self.tol is not None:
                self._inertia = float(shift)
                if self._inertia <= self.tol:
                    break
            else:
                self._inertia = shift
        if not isinstance(self._inertia, float) and self._inertia is not None:
            self._inertia = float(self._inertia)
        self._cluster_centers = DNDarray(C, C.shape, ht.types.canonical_heat_type(C.dtype), None, x.device, x.comm,
                                         True)
        lab = labels.to(torch.int64).reshape(-1, 1) if labels is not None else \
            torch.zeros((X.shape[0], 1), dtype=torch.int64, device=X.device)
        self._labels = DNDarray(lab, (x.gshape[0], 1), ht.int64, x.split, x.device, x.comm, x.balanced)
        return self
