"""
Printing of DNDarrays (reference ``heat/core/printing.py``: ``get/set_printoptions`` 20/27,
``__str__`` 61 (output on rank 0 only), edge-item gather 80-131).

Only the edge items needed for a summarised representation are gathered (one all-gather of at
most ``2 * edgeitems`` slices per dimension along the split axis), never the whole array.
"""
from __future__ import annotations

import copy

import torch

from .dndarray import DNDarray

__all__ = ["get_printoptions", "set_printoptions"]

_DEFAULT_LINEWIDTH = 120
torch.set_printoptions(profile="default", linewidth=_DEFAULT_LINEWIDTH)
_PREFIX = "DNDarray"
_INDENT = len(_PREFIX)


def get_printoptions() -> dict:
    """The current printing options as key-value pairs."""
    return copy.copy(torch._tensor_str.PRINT_OPTS.__dict__)


def set_printoptions(precision=None, threshold=None, edgeitems=None, linewidth=None, profile=None, sci_mode=None):
    """Configure printing (NumPy/PyTorch option names; heat profiles are 120 columns wide)."""
    torch.set_printoptions(precision, threshold, edgeitems, linewidth, profile, sci_mode)
    if profile in ("default", "short", "full") and linewidth is None:
        torch._tensor_str.PRINT_OPTS.linewidth = _DEFAULT_LINEWIDTH


def _torch_data(dndarray: DNDarray, summarize: bool) -> torch.Tensor:
    """The (possibly summarised) global data as a local tensor, collective."""
    if not dndarray.is_distributed():
        return dndarray.larray
    if not summarize:
        return dndarray._gathered()
    edge = torch._tensor_str.PRINT_OPTS.edgeitems
    s = dndarray.split
    t = dndarray.larray
    # reduce every summarised dimension to edge+1 leading and edge trailing items: the gathered
    # tensor stays larger than 2*edge along it, so torch's formatter still prints the "..." there
    for d in range(t.dim()):
        if d != s and t.shape[d] > 2 * edge:
            idx = torch.cat([torch.arange(edge + 1), torch.arange(t.shape[d] - edge, t.shape[d])]).to(t.device)
            t = t.index_select(d, idx)
    n = dndarray.gshape[s]
    counts, displs = dndarray.counts_displs()
    me = dndarray.comm.rank
    if n > 2 * edge:
        keep = [i for i in range(counts[me]) if displs[me] + i < edge + 1 or displs[me] + i >= n - edge]
        t = t.index_select(s, torch.tensor(keep, dtype=torch.int64, device=t.device))
    return dndarray.comm.allgather_tensor(t.contiguous(), s)


def _tensor_str(dndarray: DNDarray, indent: int) -> str:
    summarize = dndarray.gnumel > torch._tensor_str.PRINT_OPTS.threshold
    data = _torch_data(dndarray, summarize)
    if dndarray.comm.rank != 0:
        return ""
    if data.dim() == 0:
        return torch._tensor_str._scalar_str(data, torch._tensor_str._Formatter(data)) if hasattr(
            torch._tensor_str, "_scalar_str") else str(data.item())
    fmt = torch._tensor_str._Formatter(torch._tensor_str.get_summarized_data(data) if summarize else data)
    return torch._tensor_str._tensor_str_with_formatter(data, indent, summarize, fmt)


def __str__(dndarray: DNDarray) -> str:
    s = _tensor_str(dndarray, _INDENT + 1)
    if dndarray.comm.rank != 0:
        return ""
    return "{}({}, dtype=ht.{}, device={}, split={})".format(_PREFIX, s, dndarray.dtype.__name__, dndarray.device,
                                                             dndarray.split)


def __repr__(dndarray: DNDarray) -> str:
    return __str__(dndarray)
