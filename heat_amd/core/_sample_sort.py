"""
Batched distributed sample sort (parallel sorting by regular sampling) for ``sort`` /
``percentile`` / ``median`` along the split axis (reference ``core/manipulations.py:2258-2509``).

All C independent columns (every index combination of the non-split axes) are sorted together:
each step of the algorithm is ONE collective shared by all columns - two metadata all-gathers
(regular samples, partition counts) and two personalised exchanges (partitions, rebalancing) of
values + indices - whatever C is. The reference loops its Alltoallv over every column index
(``manipulations.py:2394-2411, 2469-2489``), i.e. 4*C collectives for C columns.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from .dndarray import _chunk_counts


def local_sort(t: torch.Tensor, dim: int = -1, descending: bool = False):
    """Stable ``torch.sort`` semantics; device float32 / int32 data goes to the native LSD radix
    sort (``ops.sort_rows``, csrc/radix.hip)."""
    from .. import ops

    if ops.radix_sort_supported(t, dim):
        moved = t.movedim(dim, -1)
        v, i = ops.sort_rows(moved, descending)
        return v.movedim(-1, dim), i.movedim(-1, dim)
    return torch.sort(t, dim=dim, descending=descending, stable=True)


def _overlap(lo: np.ndarray, hi: np.ndarray, a: int, b: int) -> np.ndarray:
    """Length of the intersection of every interval [lo, hi) with [a, b)."""
    return np.clip(np.minimum(hi, b) - np.maximum(lo, a), 0, None)


def _exchange_flat(comm, flat: torch.Tensor, send: List[int], recv: List[int]) -> torch.Tensor:
    parts = comm.exchange(list(torch.split(flat, send)), [(int(c),) for c in recv])
    return torch.cat(parts) if parts else flat.new_empty(0)


def sort_columns(cols: torch.Tensor, gidx: torch.Tensor, comm, n_total: int):
    """Sort every row of ``cols`` (C, nloc) across the ranks of ``comm``; ``gidx`` (nloc,) holds
    the global positions of this rank's elements. Returns (values, int64 global indices) of this
    rank's balanced block (``chunk`` rule) of every sorted column, shape (C, chunk). Stable: ties
    keep the order of their global positions."""
    p, me = comm.size, comm.rank
    C, nloc = cols.shape
    dev = cols.device
    vals, order = local_sort(cols, 1)
    idx = gidx[order]
    ar_p = torch.arange(1, p, device=dev)
    # p-1 regular samples per rank and column -> p-1 pivots per column (same on every rank)
    samples = vals[:, ((ar_p * nloc) // p).clamp(max=nloc - 1)] if nloc else vals.new_empty((C, 0))
    all_samples, _ = torch.sort(comm.allgather_tensor(samples.contiguous(), 1), dim=1)
    m = all_samples.shape[1]
    pivots = all_samples[:, ((ar_p * m) // p).clamp(max=max(m - 1, 0))].contiguous()
    # cuts[c, q]: first local position of column c that goes to rank q + 1
    cuts = torch.searchsorted(vals.contiguous(), pivots, right=True)
    edges = torch.cat([torch.zeros((C, 1), dtype=cuts.dtype, device=dev), cuts,
                       torch.full((C, 1), nloc, dtype=cuts.dtype, device=dev)], dim=1)
    send_counts = (edges[:, 1:] - edges[:, :-1]).to(torch.int64)  # (C, p)
    all_counts = comm.allgather_tensor(send_counts.unsqueeze(0).to(comm._small_device()), 0).cpu().numpy()
    # group the elements by (destination, column); stable, so every group stays sorted
    pos = torch.arange(nloc, device=dev).expand(C, nloc).contiguous()
    dest = torch.searchsorted(cuts.contiguous(), pos, right=True)
    colid = torch.arange(C, device=dev).unsqueeze(1).expand(C, nloc)
    perm = torch.sort((dest * C + colid).reshape(-1), stable=True)[1]
    send = send_counts.sum(0).tolist()
    recv_cnt = all_counts[:, :, me]  # (source rank, column)
    recv = recv_cnt.sum(1).tolist()
    mv = _exchange_flat(comm, vals.reshape(-1)[perm], send, recv)
    mi = _exchange_flat(comm, idx.reshape(-1)[perm], send, recv)
    # merge: order by (column, value); stable, so ties keep source-rank (= global position) order
    colid = torch.repeat_interleave(torch.arange(C, device=dev).repeat(p),
                                    torch.as_tensor(recv_cnt.reshape(-1), device=dev))
    mv, o = local_sort(mv)
    o2 = torch.sort(colid[o], stable=True)[1]
    mv, mi = mv[o2], mi[o[o2]]
    # rebalance: column c on rank r now holds sorted positions [start[c, r], start[c, r] + held[c, r])
    held = all_counts.sum(0)  # (C, p)
    start = np.concatenate([np.zeros((C, 1), dtype=np.int64), np.cumsum(held, axis=1)[:, :-1]], axis=1)
    tgt = _chunk_counts(n_total, p)
    bounds = np.concatenate([[0], np.cumsum(tgt)]).astype(np.int64)
    mine = held[:, me]
    colstart = np.concatenate([[0], np.cumsum(mine)[:-1]]).astype(np.int64)
    col_of = torch.repeat_interleave(torch.arange(C, device=dev), torch.as_tensor(mine, device=dev))
    g = (torch.arange(int(mine.sum()), device=dev) - torch.as_tensor(colstart, device=dev)[col_of]
         + torch.as_tensor(start[:, me], device=dev)[col_of])
    owner = torch.searchsorted(torch.as_tensor(bounds[1:], device=dev), g, right=True)
    perm = torch.sort(owner * C + col_of, stable=True)[1]
    send = [int(_overlap(start[:, me], start[:, me] + mine, bounds[q], bounds[q + 1]).sum()) for q in range(p)]
    rcol = np.stack([_overlap(start[:, q], start[:, q] + held[:, q], bounds[me], bounds[me + 1])
                     for q in range(p)])  # (source rank, column)
    recv = rcol.sum(1).tolist()
    rv = _exchange_flat(comm, mv[perm], send, recv)
    ri = _exchange_flat(comm, mi[perm], send, recv)
    # received by source rank, each block grouped by column: a stable column sort restores order
    cid = torch.repeat_interleave(torch.arange(C, device=dev).repeat(p), torch.as_tensor(rcol.reshape(-1), device=dev))
    o = torch.sort(cid, stable=True)[1]
    nme = tgt[me]
    return rv[o].reshape(C, nme), ri[o].reshape(C, nme)
