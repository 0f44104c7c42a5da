"""
Ring pipeline primitive (the reference's "ring pass" in ``spatial/distance.py:265-362, 429-486``
and ``linalg/basics.py:1232-1266``).

``ring_pass(block, fn, comm)`` calls ``fn(moving_block, source_rank)`` for every rank's block,
starting with the local one, while the next block is already in flight (double-buffered batched
isend/irecv to the ring neighbours), so communication overlaps the compute of ``fn``.
"""
from __future__ import annotations

from typing import Callable, List

import torch
import torch.distributed as dist

from . import staging as _SD


def ring_pass(block: torch.Tensor, fn: Callable[[torch.Tensor, int], None], comm, sizes: List[int] = None):
    """Visit every rank's ``block`` in ring order (own first), overlapping transfer and compute.

    ``sizes`` (optional) gives every rank's leading dimension when blocks are uneven."""
    p, me = comm.size, comm.rank
    if p == 1:
        fn(block, me)
        return
    if sizes is None:
        sizes = comm.allgather_sizes(block.shape[0])
    rest = tuple(block.shape[1:])
    cur = block.contiguous()
    src = me
    nxt, prv = (me + 1) % p, (me - 1) % p
    for step in range(p):
        works = []
        recv = None
        if step < p - 1:
            incoming = (me - step - 1) % p
            recv = torch.empty((sizes[incoming],) + rest, dtype=cur.dtype, device=cur.device)
            ops = [dist.P2POp(dist.isend, cur, comm._g(nxt), comm.group),
                   dist.P2POp(dist.irecv, recv, comm._g(prv), comm.group)]
            works = _SD.batch_isend_irecv(ops)
        fn(cur, src)
        for w in works:
            w.wait()
        if recv is not None:
            cur = recv
            src = (src - 1) % p
