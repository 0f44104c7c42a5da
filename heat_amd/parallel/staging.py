"""
Device-buffer staging for process groups that cannot take device tensors (the
reference's non-CUDA-aware MPI path ``communication.py:16-26`` and its ``.cpu()`` copies).

With RCCL (``cuda:nccl`` in the default mixed group) device tensors go straight onto xGMI and
nothing here does anything. With a pure ``gloo`` group - CPU tests, or several ranks sharing one
GPU where RCCL refuses a duplicate device - a device tensor is copied to host memory, the
collective runs there and the result is copied back when the work completes. The wrappers keep
the ``torch.distributed`` signatures and the asynchronous ``work.wait()`` contract, so the
communication layer issues every collective through them unconditionally.
"""
from __future__ import annotations

import os
from typing import List

import torch
import torch.distributed as dist

_BACKEND_CACHE = {}
# tests: stage host tensors too, so CPU runs exercise every wrapper's copy-in / copy-back path
_FORCE = os.environ.get("HEAT_COMM_FORCE_STAGING", "0") == "1"


def _backend(group) -> str:
    key = id(group) if group is not None else None
    b = _BACKEND_CACHE.get(key)
    if b is None:
        b = str(dist.get_backend(group))
        _BACKEND_CACHE[key] = b
    return b


def needs_staging(group, *tensors) -> bool:
    """True for device tensors on a group whose backend is gloo only."""
    if _FORCE:
        return True
    if not any(t is not None and t.is_cuda for t in tensors):
        return False
    return _backend(group) == "gloo"


class StagedWork:
    """``work.wait()`` that also copies staged results back into the device buffers."""

    def __init__(self, work, fin=None):
        self._work = work
        self._fin = fin
        self._done = False

    def wait(self, timeout=None):
        if not self._done:
            if self._work is not None:
                self._work.wait()
            if self._fin is not None:
                self._fin()
            self._done = True
        return True

    def is_completed(self) -> bool:
        return self._done or self._work is None or self._work.is_completed()


def _host(t):
    return t.detach().to("cpu", copy=True)


def _ret(work, fin, async_op):
    w = StagedWork(work, fin)
    if async_op:
        return w
    w.wait()
    return None


def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
    """``dist.all_reduce``; for a gloo group and device tensor the data goes through a host copy."""
    if not needs_staging(group, t):
        return dist.all_reduce(t, op=op, group=group, async_op=async_op)
    h = _host(t)
    work = dist.all_reduce(h, op=op, group=group, async_op=True)
    return _ret(work, lambda: t.copy_(h), async_op)


def broadcast(t, src, group=None, async_op=False):
    """``dist.broadcast`` with host staging for gloo groups and device tensors."""
    if not needs_staging(group, t):
        return dist.broadcast(t, src=src, group=group, async_op=async_op)
    h = _host(t)
    work = dist.broadcast(h, src=src, group=group, async_op=True)
    return _ret(work, lambda: t.copy_(h), async_op)


def all_gather_into_tensor(out, inp, group=None, async_op=False):
    """``dist.all_gather_into_tensor`` with host staging for gloo groups and device tensors."""
    if not needs_staging(group, out, inp):
        return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)
    ho = torch.empty(out.shape, dtype=out.dtype)
    work = dist.all_gather_into_tensor(ho, _host(inp), group=group, async_op=True)
    return _ret(work, lambda: out.copy_(ho), async_op)


def reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=None, async_op=False):
    """``dist.reduce_scatter_tensor``; gloo has none, so a staged all-reduce keeps this rank's slice."""
    if not needs_staging(group, out, inp):
        return dist.reduce_scatter_tensor(out, inp, op=op, group=group, async_op=async_op)
    # gloo has no reduce_scatter of flat tensors: all-reduce the whole input, keep this rank's part
    h = _host(inp)
    work = dist.all_reduce(h, op=op, group=group, async_op=True)
    rank = dist.get_rank(group)
    n = out.numel()
    return _ret(work, lambda: out.copy_(h.reshape(-1)[rank * n:(rank + 1) * n].reshape(out.shape)), async_op)


def all_to_all_single(out, inp, out_split_sizes=None, in_split_sizes=None, group=None, async_op=False):
    """``dist.all_to_all_single`` with host staging for gloo groups and device tensors."""
    if not needs_staging(group, out, inp):
        return dist.all_to_all_single(out, inp, out_split_sizes, in_split_sizes, group=group, async_op=async_op)
    ho = torch.empty(out.shape, dtype=out.dtype)
    work = dist.all_to_all_single(ho, _host(inp), out_split_sizes, in_split_sizes, group=group, async_op=True)
    return _ret(work, lambda: out.copy_(ho), async_op)


def isend(t, dst, group=None, tag=0):
    """``dist.isend``; a staged send keeps its host copy alive in the returned work object."""
    if not needs_staging(group, t):
        return dist.isend(t, dst=dst, group=group, tag=tag)
    h = _host(t)
    return StagedWork(dist.isend(h, dst=dst, group=group, tag=tag), lambda: h)


def irecv(t, src, group=None, tag=0):
    """``dist.irecv``; a staged receive copies into ``t`` when its work object is waited on."""
    if not needs_staging(group, t):
        return dist.irecv(t, src=src, group=group, tag=tag)
    h = torch.empty(t.shape, dtype=t.dtype)
    return StagedWork(dist.irecv(h, src=src, group=group, tag=tag), lambda: t.copy_(h))


def recv(t, src, group=None, tag=0):
    """Blocking receive into ``t`` (staged as ``irecv``)."""
    irecv(t, src, group, tag).wait()


def batch_isend_irecv(ops: List["dist.P2POp"]):
    """``dist.batch_isend_irecv`` with host staging for gloo groups and device tensors; the
    received host buffers are copied back when the returned works are waited on."""
    if not ops or not needs_staging(ops[0].group, *[o.tensor for o in ops]):
        return dist.batch_isend_irecv(ops)
    staged, fins = [], []
    for o in ops:
        if o.op in (dist.isend, dist.send) or getattr(o.op, "__name__", "") in ("isend", "send"):
            staged.append(dist.P2POp(dist.isend, _host(o.tensor), o.peer, o.group, o.tag))
            fins.append(None)
        else:
            h = torch.empty(o.tensor.shape, dtype=o.tensor.dtype)
            staged.append(dist.P2POp(dist.irecv, h, o.peer, o.group, o.tag))
            fins.append((o.tensor, h))
    works = dist.batch_isend_irecv(staged)

    def mk(w, f):
        return StagedWork(w, (lambda: f[0].copy_(f[1])) if f is not None else None)

    return [mk(w, f) for w, f in zip(works, fins)]
