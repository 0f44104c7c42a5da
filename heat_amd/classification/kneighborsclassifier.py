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
                if kk:
                    vals, idx = torch.topk(d, kk, dim=1, largest=False)
                    cand_y = ylab[idx.reshape(-1).to(ylab.device)].reshape(d.shape[0], kk, -1)
                else:
                    vals = d.new_zeros((d.shape[0], 0))
                    cand_y = ylab.new_zeros((d.shape[0], 0, ylab.shape[1]))
                comm = distances.comm
                all_v = comm.allgather_tensor(vals.to(torch.float64).contiguous(), 1)
                all_y = comm.allgather_tensor(cand_y.contiguous(), 1)
                _, sel = torch.topk(all_v, k, dim=1, largest=False)
                votes = torch.gather(all_y, 1, sel.unsqueeze(-1).expand(-1, -1, all_y.shape[-1])).sum(1)
            else:
                d = distances.larray
                _, idx = torch.topk(d, k, dim=1, largest=False)
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
        best_y = torch.zeros((nq, k, ylab.shape[1]), dtype=torch.float32, device=q.device)
        if train.is_distributed():
            packed = torch.cat([tl.float(), ylab], dim=1)
            counts = train.split_counts()

            def visit(block: torch.Tensor, src: int):
                _merge(block[:, : tl.shape[1]], block[:, tl.shape[1]:])

        def _merge(tb: torch.Tensor, yb: torch.Tensor):
            nonlocal best_d, best_y
            if tb.shape[0] == 0 or nq == 0:
                return
            # fused distance + running top-k kernel (no nq x nt matrix); exact distances of the picks
            kk = min(k, tb.shape[0])
            dv, di = ops.knn_topk(q.float(), tb.float(), kk)
            cand_d = torch.cat([best_d, dv], dim=1)
            cand_y = torch.cat([best_y, yb[di.reshape(-1)].reshape(nq, kk, -1)], dim=1)
            sel_d, sel = torch.topk(cand_d, k, dim=1, largest=False)
            best_d = sel_d
            best_y = torch.gather(cand_y, 1, sel.unsqueeze(2).expand(-1, -1, cand_y.shape[2]))

        if train.is_distributed():
            ring_pass(packed, visit, train.comm, counts)
        else:
            _merge(tl.float(), ylab)
        votes = best_y.sum(1)
        lab = torch.argmax(votes, dim=1)
        self.classes_ = DNDarray(lab, (x.gshape[0],), ht.int64, x.split, x.device, x.comm, x.balanced)
        return self.classes_
