"""Graph Laplacian from a dataset (reference ``heat/graph/laplacian.py``: ``Laplacian`` 12,
``_normalized_symmetric_L`` 73, ``_simple_L`` 97, ``construct`` 112)."""
from __future__ import annotations

from typing import Callable

import torch

from .. import core as ht
from ..core.dndarray import DNDarray

__all__ = ["Laplacian"]


class Laplacian:
    """Graph Laplacian (``definition`` 'simple' or 'norm_sym'; ``mode`` 'fully_connected' or
    'eNeighbour' with an upper/lower similarity threshold)."""

    def __init__(self, similarity: Callable, weighted: bool = True, definition: str = "norm_sym",
                 mode: str = "fully_connected", threshold_key: str = "upper", threshold_value: float = 1.0,
                 neighbours: int = 10):
        self.similarity_metric = similarity
        self.weighted = weighted
        if definition not in ("simple", "norm_sym"):
            raise NotImplementedError("Currently only simple and normalized symmetric graph laplacians are supported")
        self.definition = definition
        if mode not in ("eNeighbour", "fully_connected"):
            raise NotImplementedError("Only eNeighborhood and fully-connected graphs supported at the moment.")
        self.mode = mode
        if threshold_key not in ("upper", "lower"):
            raise ValueError("Only 'upper' and 'lower' threshold types supported for eNeighbouhood graph construction")
        self.epsilon = (threshold_key, threshold_value)
        self.neighbours = neighbours

    def _normalized_symmetric_L(self, A: DNDarray) -> DNDarray:
        """``L = I - D^-1/2 A D^-1/2`` (isolated vertices get degree 1)."""
        degree = ht.sum(A, axis=1)
        degree = ht.resplit(degree, None)
        d = degree.larray
        d = torch.where(d == 0, torch.ones_like(d), d)
        inv = torch.rsqrt(d)
        t = A.larray
        if A.is_distributed():
            counts, displs = A.counts_displs()
            r = A.comm.rank
            if A.split == 0:
                rows = inv[displs[r]: displs[r] + counts[r]]
                cols = inv
            else:
                rows = inv
                cols = inv[displs[r]: displs[r] + counts[r]]
        else:
            rows = cols = inv
        L = -(t * rows.unsqueeze(1) * cols.unsqueeze(0))
        res = DNDarray(L, A.gshape, A.dtype, A.split, A.device, A.comm, A.balanced)
        res.fill_diagonal(1.0)
        return res

    def _simple_L(self, A: DNDarray) -> DNDarray:
        """``L = D - A``."""
        degree = ht.sum(A, axis=1)
        return ht.diag(degree) - A

    def construct(self, X: DNDarray) -> DNDarray:
        """Laplacian of the similarity graph of the rows of X."""
        S = self.similarity_metric(X)
        S.fill_diagonal(0.0)
        if self.mode == "eNeighbour":
            key, val = self.epsilon
            t = S.larray
            if key == "upper":
                mask = t < val
            else:
                mask = t > val
            if self.weighted:
                S.larray = torch.where(mask, t, torch.zeros_like(t))
            else:
                S.larray = mask.to(t.dtype)
        if self.definition == "simple":
            return self._simple_L(S)
        return self._normalized_symmetric_L(S)
