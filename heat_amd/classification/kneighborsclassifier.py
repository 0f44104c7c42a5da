"""
k-nearest-neighbours classifier (reference ``heat/classification/kneighborsclassifier.py``:
``KNeighborsClassifier`` 9, ``one_hot_encoding`` 45, ``fit`` 62, ``predict`` 117).

The reference materialises the full query x training distance matrix, runs a distributed top-k
and gathers one-hot labels. Here every rank streams the training blocks around a double-buffered
ring (``parallel.ring_pass``), computes one distance tile at a time with the native kernel and
keeps a running per-query top-k: memory O(m_local * (k + block)), no distance matrix.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from .. import core as ht
from ..core.base import BaseEstimator, ClassificationMixin
from ..core.dndarray import DNDarray
from .. import ops
from ..parallel.ring import ring_pass

__all__ = ["KNeighborsClassifier"]


def _smallest_k(vals: torch.Tensor, gidx: torch.Tensor, k: int) -> torch.Tensor:
    """Positions (along dim 1) of the ``k`` smallest ``vals``, equal values ordered by global
    training index ``gidx``: two stable sorts, so the pick does not depend on the visiting order of
    the blocks (and thus not on the number of ranks)."""
    o1 = torch.sort(gidx, dim=1, stable=True).indices
    o2 = torch.sort(torch.gather(vals, 1, o1), dim=1, stable=True).indices
    return torch.gather(o1, 1, o2[:, :k])


class KNeighborsClassifier(ClassificationMixin, BaseEstimator):
    """Majority vote of the ``n_neighbors`` nearest training samples (euclidean by default)."""

    def __init__(self, n_neighbors: int = 5, effective_metric_: Callable = None):
        self.n_neighbors = n_neighbors
        self.effective_metric_ = effective_metric_

    @staticmethod
    def one_hot_encoding(x: DNDarray) -> DNDarray:
        """One-hot encode integer labels (classes 0 .. max)."""
        n_features = int(ht.max(x).item()) + 1
        t = x.larray.to(torch.int64)
        one_hot = torch.zeros((t.shape[0], n_features), dtype=torch.float32, device=t.device)
        one_hot.scatter_(1, t.reshape(-1, 1), 1.0)
        return DNDarray(one_hot, (x.gshape[0], n_features), ht.float32, x.split, x.device, x.comm, x.balanced)

    def fit(self, x: DNDarray, y: DNDarray) -> "KNeighborsClassifier":
        if not isinstance(x, DNDarray) or not isinstance(y, DNDarray):
            raise TypeError("x and y must be DNDarrays but were {} {}".format(type(x), type(y)))
        if x.ndim != 2:
            raise ValueError("x must be two-dimensional, but was {}".format(x.ndim))
        if x.gshape[0] != y.gshape[0]:
            raise ValueError("Number of samples x and y samples mismatch, got {}, {}".format(x.gshape[0], y.gshape[0]))
        if y.split != x.split and x.comm.size > 1:
            # labels travel with their samples: y takes x's distribution
            y = ht.resplit(y, x.split if x.split == 0 else None)
        if x.split == 0 and y.split == 0 and x.is_distributed():
            xmap = x.create_lshape_map()
            ymap = y.create_lshape_map()
            if not torch.equal(xmap[:, 0], ymap[:, 0]):
                # same split, different row blocks (e.g. an unbalanced x): move y's rows to x's
                y = y.copy()
                target = ymap.clone()
                target[:, 0] = xmap[:, 0]
                y.redistribute_(lshape_map=ymap, target_map=target)
        self.x = x
        self.n_samples_fit_ = x.gshape[0]
        if y.ndim == 1:
            self.y = self.one_hot_encoding(y)
            self.outputs_2d_ = False
        elif y.ndim == 2:
            self.y = y
            self.outputs_2d_ = True
        else:
            raise ValueError("y needs to be one- or two-dimensional, but was {}".format(y.ndim))
        return self

    def predict(self, x: DNDarray) -> DNDarray:
        k = self.n_neighbors
        if self.effective_metric_ is not None:
            distances = self.effective_metric_(x, self.x)
            if distances.split == 1 and distances.is_distributed():
                # columns = training rows, split like the labels: local top-k of every rank's
                # column block, ONE all-gather of the p x k candidates (distance + label vector),
                # top-k of those - the query x train matrix is never gathered
                d = distances.larray
                kk = min(k, d.shape[1])
                ylab = self.y.larray.to(torch.float32)
                comm = distances.comm
                col0 = sum(distances.split_counts()[: comm.rank])
                if ylab.shape[0] != d.shape[1]:
                    raise ValueError("distance columns ({}) and local labels ({}) are not aligned".format(
                        d.shape[1], ylab.shape[0]))
                if kk:
                    cols = torch.arange(d.shape[1], device=d.device).expand(d.shape[0], -1)
                    idx = _smallest_k(d, cols, kk)
                    vals = torch.gather(d, 1, idx)
                    cand_y = ylab[idx.reshape(-1).to(ylab.device)].reshape(d.shape[0], kk, -1)
                else:
                    idx = torch.zeros((d.shape[0], 0), dtype=torch.int64, device=d.device)
                    vals = d.new_zeros((d.shape[0], 0))
                    cand_y = ylab.new_zeros((d.shape[0], 0, ylab.shape[1]))
                all_v = comm.allgather_tensor(vals.to(torch.float64).contiguous(), 1)
                all_i = comm.allgather_tensor((idx + col0).to(torch.int64).contiguous(), 1)
                all_y = comm.allgather_tensor(cand_y.contiguous(), 1)
                sel = _smallest_k(all_v, all_i, k)
                votes = torch.gather(all_y, 1, sel.unsqueeze(-1).expand(-1, -1, all_y.shape[-1])).sum(1)
            else:
                d = distances.larray
                idx = _smallest_k(d, torch.arange(d.shape[1], device=d.device).expand(d.shape[0], -1), k)
                ylab = self.y._gathered() if self.y.is_distributed() else self.y.larray
                votes = ylab[idx.reshape(-1).to(ylab.device)].reshape(idx.shape[0], k, -1).sum(1)
            lab = torch.argmax(votes, dim=1)
            return DNDarray(lab, (x.gshape[0],), ht.int64, x.split if x.split == 0 else None, x.device, x.comm,
                            x.balanced)
        q = x.larray if x.larray.is_floating_point() else x.larray.float()
        train = self.x
        tl = train.larray.to(q.dtype)
        ylab = self.y.larray.to(torch.float32)
        nq = q.shape[0]
        best_d = torch.full((nq, k), float("inf"), dtype=torch.float32, device=q.device)
        best_i = torch.full((nq, k), torch.iinfo(torch.int64).max, dtype=torch.int64, device=q.device)
        best_y = torch.zeros((nq, k, ylab.shape[1]), dtype=torch.float32, device=q.device)
        if train.is_distributed():
            if ylab.shape[0] != tl.shape[0]:
                raise ValueError("training rows ({}) and local labels ({}) are not aligned".format(
                    tl.shape[0], ylab.shape[0]))
            packed = torch.cat([tl.float(), ylab], dim=1)
            counts = train.split_counts()
            starts = [sum(counts[:r]) for r in range(len(counts))]

            def visit(block: torch.Tensor, src: int):
                _merge(block[:, : tl.shape[1]], block[:, tl.shape[1]:], starts[src])

        def _merge(tb: torch.Tensor, yb: torch.Tensor, row0: int):
            nonlocal best_d, best_i, best_y
            if tb.shape[0] == 0 or nq == 0:
                return
            # fused distance + running top-k kernel (no nq x nt matrix); exact distances of the picks
            kk = min(k, tb.shape[0])
            dv, di = ops.knn_topk(q.float(), tb.float(), kk)
            cand_d = torch.cat([best_d, dv], dim=1)
            cand_i = torch.cat([best_i, di.to(torch.int64) + row0], dim=1)
            cand_y = torch.cat([best_y, yb[di.reshape(-1)].reshape(nq, kk, -1)], dim=1)
            sel = _smallest_k(cand_d, cand_i, k)   # ties by global training index
            best_d = torch.gather(cand_d, 1, sel)
            best_i = torch.gather(cand_i, 1, sel)
            best_y = torch.gather(cand_y, 1, sel.unsqueeze(2).expand(-1, -1, cand_y.shape[2]))

        if train.is_distributed():
            ring_pass(packed, visit, train.comm, counts)
        else:
            _merge(tl.float(), ylab, 0)
        votes = best_y.sum(1)
        lab = torch.argmax(votes, dim=1)
        self.classes_ = DNDarray(lab, (x.gshape[0],), ht.int64, x.split, x.device, x.comm, x.balanced)
        return self.classes_
