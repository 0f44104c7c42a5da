"""
Ring pipeline primitive (the reference's "ring pass" in ``spatial/distance.py:265-362, 429-486``
and ``linalg/basics.py:1232-1266``).

``ring_pass(block, fn, comm)`` calls ``fn(moving_block, source_rank)`` for every rank's block,
starting with the local one, while the next block is already in flight (double-buffered batched
isend/irecv to the ring neighbours), so communication overlaps the compute of ``fn``.
"""
from __future__ import annotations

import os
from collections import Counter
from typing import Callable, List

import torch
import torch.distributed as dist

from . import staging as _SD


#: passes taken per mode ("ring" / "direct"), reported by ``bench.py``
PASSES = Counter()


def ring_mode() -> str:
    """``HEAT_RING_MODE``: "ring" (default: two blocks in memory, one neighbour link per step) or
    "direct" (every rank posts its block to all p - 1 peers at once - on a fully connected xGMI node
    all 7 links of a GPU carry data concurrently - and the blocks are consumed in ring order as they
    arrive; p blocks in memory)."""
    return os.environ.get("HEAT_RING_MODE", "ring")


def ring_pass(block: torch.Tensor, fn: Callable[[torch.Tensor, int], None], comm, sizes: List[int] = None,
              mode: str = None):
    """Visit every rank's ``block`` in ring order (own first), overlapping transfer and compute.

    ``sizes`` (optional) gives every rank's leading dimension when blocks are uneven; ``mode``
    overrides :func:`ring_mode`."""
    p, me = comm.size, comm.rank
    if p == 1:
        fn(block, me)
        return
    if sizes is None:
        sizes = comm.allgather_sizes(block.shape[0])
    if (mode or ring_mode()) == "direct":
        PASSES["direct"] += 1
        return _direct_pass(block, fn, comm, sizes)
    PASSES["ring"] += 1
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


def _direct_pass(block: torch.Tensor, fn, comm, sizes: List[int]):
    """All-peers variant of :func:`ring_pass`: one batched group of p - 1 sends of the local block
    and p - 1 receives (pairwise order: step k sends to rank + k and receives from rank - k, so
    every link is busy in both directions), then ``fn`` on the own block while the transfers run,
    then on every received block in ring order."""
    p, me = comm.size, comm.rank
    rest = tuple(block.shape[1:])
    cur = block.contiguous()
    recvs, ops = {}, []
    for k in range(1, p):
        to, frm = (me + k) % p, (me - k) % p
        recvs[frm] = torch.empty((sizes[frm],) + rest, dtype=cur.dtype, device=cur.device)
        ops.append(dist.P2POp(dist.isend, cur, comm._g(to), comm.group))
        ops.append(dist.P2POp(dist.irecv, recvs[frm], comm._g(frm), comm.group))
    works = _SD.batch_isend_irecv(ops)
    fn(cur, me)
    for w in works:
        w.wait()
    for k in range(1, p):
        src = (me - k) % p
        fn(recvs.pop(src), src)
