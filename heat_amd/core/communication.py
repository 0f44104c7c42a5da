"""
Split-tensor communication layer over ``torch.distributed`` (RCCL over xGMI for device buffers,
gloo for host buffers).

API parity with the reference's ``heat/core/communication.py`` (``MPIRequest`` 29,
``MPICommunication`` 120, ``chunk`` 161, ``counts_displs_shape`` 211, p2p 439-668, ``Bcast`` 697,
``Allreduce`` 789, ``Exscan`` 814, ``Allgather(v)`` 1074/1103, ``Alltoall(v)`` 1324/1360,
``Gather(v)/Scatter(v)`` 1557-1853, ``MPI_WORLD/MPI_SELF`` 1867, ``use_comm`` 1904): the same
method names, the same buffer conventions (torch tensors or DNDarrays, ``(buf, counts, displs)``
tuples for v-variants, ``MPI.IN_PLACE``) and the same axis semantics.

The implementation is MI355X-first rather than an MPI emulation:

* RCCL has no tags, probes, v-collectives, scans, custom ops or derived datatypes. v-collectives
  are a single ``all_to_all_single`` (grouped point-to-point inside RCCL) on a packed buffer, or a
  pad-to-max ``all_gather_into_tensor`` for Allgatherv (one collective, all 7 xGMI links busy).
* Custom reduction ops (argmax/argmin pairs, top-k merge, bf16 sums) are an all-gather of the p
  partials followed by an on-device fold - p <= 8 on one node, so this is one small collective
  instead of p log p point-to-point hops.
* Scans are an all-gather of one slice per rank plus a local prefix.
* Strided sub-tensors are packed contiguously on the device (``narrow().contiguous()``) instead of
  MPI derived datatypes.
* Device buffers go straight to RCCL. Only a pure gloo group (``HEAT_COMM_BACKEND=gloo``: CPU
  tests, or several ranks sharing one GPU) stages them through host memory
  (``parallel/staging.py``, the reference's non-CUDA-aware path); ``CUDA_AWARE_MPI`` says which.
"""
from __future__ import annotations

import os
import pickle
from collections import Counter
from typing import Any, Callable, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.distributed as dist

from ..parallel import backend as _backend
from ..parallel import staging as _SD

# device buffers are handed straight to RCCL unless the world group is gloo-only (host staging)
CUDA_AWARE_MPI = _backend.backend_name() != "gloo"

#: collective -> data path counters ("allreduce:ipc", "allreduce:native", "allreduce:pg",
#: "allgatherv:...", "reduce_scatter:..."); ``bench.py`` reports them so a run records which
#: path (torch ProcessGroup / native RCCL communicator / xGMI IPC kernels) each collective took
PATH_COUNTS = Counter()


# ----------------------------------------------------------------------------------------------
# MPI-flavoured constants and ops (user code and tests reference ``MPI.SUM`` etc.)
# ----------------------------------------------------------------------------------------------
class _InPlace:
    def __repr__(self):
        return "MPI.IN_PLACE"


class Op:
    """A reduction operator. Built-ins map to RCCL reductions; custom ops fold all-gathered partials."""

    def __init__(self, name: str, torch_op=None, fold: Optional[Callable] = None, commute: bool = True):
        self.name = name
        self.torch_op = torch_op
        self.fold = fold
        self.commute = commute

    @classmethod
    def Create(cls, function: Callable, commute: bool = True) -> "Op":
        """Create a custom op from ``function(a, b) -> reduced`` acting on torch tensors.

        For compatibility with mpi4py-style callbacks ``function(inbuf, inoutbuf, datatype)`` that
        write into ``inoutbuf``, a three-argument callback is also accepted.
        """
        import inspect

        try:
            nargs = len(inspect.signature(function).parameters)
        except (TypeError, ValueError):
            nargs = 2
        if nargs >= 3:
            def fold(a, b, _f=function):
                out = b.clone()
                _f(a, out, None)
                return out
        else:
            fold = function
        return cls("custom", None, fold, commute)

    def Free(self):
        pass

    def __repr__(self):
        return "MPI.{}".format(self.name)


def _band(a, b):
    return a & b


def _bor(a, b):
    return a | b


def _bxor(a, b):
    return a ^ b


class MPI:
    """Namespace mirroring the mpi4py names the heat API exposes."""

    IN_PLACE = _InPlace()
    SUM = Op("SUM", dist.ReduceOp.SUM, torch.add)
    PROD = Op("PROD", dist.ReduceOp.PRODUCT, torch.mul)
    MIN = Op("MIN", dist.ReduceOp.MIN, torch.minimum)
    MAX = Op("MAX", dist.ReduceOp.MAX, torch.maximum)
    LAND = Op("LAND", None, torch.logical_and)
    LOR = Op("LOR", None, torch.logical_or)
    LXOR = Op("LXOR", None, torch.logical_xor)
    BAND = Op("BAND", None, _band)
    BOR = Op("BOR", None, _bor)
    BXOR = Op("BXOR", None, _bxor)
    Op = Op
    ANY_SOURCE = -1
    ANY_TAG = -1
    UNDEFINED = -32766

    class Exception(RuntimeError):
        pass

    class Status:
        def __init__(self):
            self.source = None
            self.tag = None
            self.count = None

        def Get_source(self):
            return self.source

        def Get_tag(self):
            return self.tag


# ----------------------------------------------------------------------------------------------
# requests
# ----------------------------------------------------------------------------------------------
class MPIRequest:
    """Handle on a non-blocking operation. ``Wait()`` completes the work and runs the epilogue
    (copy-back into the user's receive buffer, un-permutation, custom-op fold)."""

    def __init__(self, works=None, finalize: Optional[Callable] = None, result=None):
        if works is None:
            works = []
        elif not isinstance(works, (list, tuple)):
            works = [works]
        self.handle = self
        self._works = list(works)
        self._finalize = finalize
        self._done = False
        self.result = result

    def Wait(self, status=None):
        if self._done:
            return self.result
        for w in self._works:
            if w is not None:
                w.wait()
        if self._finalize is not None:
            r = self._finalize()
            if r is not None:
                self.result = r
        self._done = True
        return self.result

    wait = Wait

    def Test(self, status=None) -> bool:
        if self._done:
            return True
        if all(w is None or w.is_completed() for w in self._works):
            self.Wait()
            return True
        return False

    test = Test

    @staticmethod
    def Waitall(requests):
        for r in requests:
            if r is not None:
                r.Wait()


# ----------------------------------------------------------------------------------------------
# communicators
# ----------------------------------------------------------------------------------------------
class Communication:
    """Base class for communicators (kept for API parity and alternative backends)."""

    @staticmethod
    def is_distributed() -> bool:
        raise NotImplementedError()

    def __init__(self):
        raise NotImplementedError()

    def chunk(self, shape, split):
        raise NotImplementedError()


def exchange_axis_bytes(send_shape, send_axis: int, scounts, recv_shape, recv_axis: int, rcounts, itemsize: int):
    """Byte counts of the packed blocks of :meth:`MPICommunication.exchange_axis`: (to every rank,
    from every rank). Block q of the send side is ``send.narrow(send_axis, ., scounts[q])`` packed
    contiguously, block r of the receive side ``recv.narrow(recv_axis, ., rcounts[r])``."""
    from ..ops import kernels as _k

    so, _, sr = _k._rows_view(tuple(send_shape), send_axis)
    ro, _, rr = _k._rows_view(tuple(recv_shape), recv_axis)
    return ([so * int(c) * sr * itemsize for c in scounts], [ro * int(c) * rr * itemsize for c in rcounts])


def _as_tensor(buf):
    from .dndarray import DNDarray

    if isinstance(buf, DNDarray):
        return buf.larray
    return buf


# dtypes neither gloo nor RCCL move: bool travels as uint8, int16 as int32 (cast back on arrival)
_WIRE = {torch.bool: torch.uint8, torch.int16: torch.int32}


def _wire_dtype(t: torch.Tensor) -> torch.Tensor:
    w = _WIRE.get(t.dtype)
    return t.to(w) if w is not None else t


class MPICommunication(Communication):
    """A communicator over a ``torch.distributed`` process group (or a world of one).

    ``group`` is a ProcessGroup (``None`` = world) and ``ranks`` the global ranks of its members.
    A communicator of size one (``MPI_SELF`` or a single-process run) performs every operation
    locally without touching ``torch.distributed``.
    """

    def __init__(self, group=None, ranks: Optional[Sequence[int]] = None, _self_only: bool = False):
        self._self_only = _self_only
        if _self_only or not _backend.ensure_initialized():
            self.group = None
            self._ranks = [dist.get_rank() if (dist.is_available() and dist.is_initialized()) else 0]
            self.rank = 0
            self.size = 1
            self._self_only = True
        else:
            self.group = group
            if ranks is None:
                ranks = list(range(dist.get_world_size()))
            self._ranks = list(ranks)
            grank = dist.get_rank()
            self.rank = self._ranks.index(grank) if grank in self._ranks else None
            self.size = len(self._ranks)
        self.handle = self
        self._debug = os.environ.get("HEAT_DEBUG_COLLECTIVES", "0") == "1"

    # ---------------------------------------------------------------- basics
    def is_distributed(self) -> bool:
        return self.size > 1

    def Get_rank(self) -> int:
        return self.rank

    def Get_size(self) -> int:
        return self.size

    def _g(self, r: int) -> int:
        """group rank -> global rank."""
        return self._ranks[r]

    def __repr__(self):
        return "MPICommunication(rank={}, size={})".format(self.rank, self.size)

    def chunk(self, shape, split, rank: int = None, w_size: int = None, sparse: bool = False):
        """Block distribution of ``shape`` along ``split``: the first ``shape[split] % p`` ranks
        hold one extra element (reference communication.py:161-209).

        Returns ``(offset, local_shape, slices)``.
        """
        from .stride_tricks import sanitize_axis

        split = sanitize_axis(shape, split)
        if split is None:
            return 0, tuple(shape), tuple(slice(0, end) for end in shape)
        rank = self.rank if rank is None else rank
        w_size = self.size if w_size is None else w_size
        n = shape[split]
        base, rem = divmod(n, w_size)
        count = base + (1 if rank < rem else 0)
        start = rank * base + min(rank, rem)
        lshape = tuple(count if i == split else s for i, s in enumerate(shape))
        slices = tuple(slice(start, start + count) if i == split else slice(0, s)
                       for i, s in enumerate(shape))
        return start, lshape, slices

    def counts_displs_shape(self, shape, axis):
        """Counts/displacements of the regular chunking of ``shape`` along ``axis`` and the output
        shape of an all-to-all receive buffer (reference communication.py:211-240)."""
        n = shape[axis]
        base, rem = divmod(n, self.size)
        counts = tuple(base + (1 if r < rem else 0) for r in range(self.size))
        displs = tuple(int(x) for x in np.concatenate(([0], np.cumsum(counts[:-1]))))
        out = list(shape)
        out[axis] = self.size * counts[self.rank]
        return counts, displs, tuple(out)

    def _check_stream(self, name, t):
        """HEAT_DEBUG_STREAMS=1: a collective on a device tensor must be issued on
        the stream the native kernels last launched on, or after that stream has drained;
        otherwise RCCL (ordered behind the CURRENT stream) may read data a kernel on the other
        stream has not written yet."""
        from .. import ops

        if not (ops.DEBUG_STREAMS and isinstance(t, torch.Tensor) and t.is_cuda):
            return
        last = ops.LAST_LAUNCH_STREAM.get(t.device.index)
        cur = torch.cuda.current_stream(t.device)
        if last is not None and last != cur and not last.query():
            raise RuntimeError("stream-ordering race: {} issued on stream {} while native kernels on stream {} are "
                               "still running; synchronise the streams (e.g. cur.wait_stream(other)) first"
                               .format(name, cur.cuda_stream, last.cuda_stream))

    def _trace(self, name, t=None):
        self._check_stream(name, t)
        if self._debug and self.size > 1:
            sig = "{}|{}|{}".format(name, None if t is None else t.dtype,
                                    None if t is None else tuple(t.shape) if name.startswith(("All", "Bcast")) else "")
            sigs = [None] * self.size
            dist.all_gather_object(sigs, sig, group=self.group)
            base = [s.split("|")[0] for s in sigs]
            if len(set(base)) != 1:
                raise RuntimeError("collective mismatch across ranks: {}".format(sigs))

    # ---------------------------------------------------------------- barrier
    def Barrier(self):
        if self.size > 1:
            if dist.get_backend(self.group) == "nccl" and torch.cuda.is_available():
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)

    barrier = Barrier

    # ---------------------------------------------------------------- broadcast
    def Ibcast(self, buf, root: int = 0) -> MPIRequest:
        t = _as_tensor(buf)
        self._trace("Bcast", t)
        if self.size == 1:
            return MPIRequest()
        wire = _wire_dtype(t)
        contig = wire if wire.is_contiguous() and wire is t else wire.contiguous()
        work = _SD.broadcast(contig, src=self._g(root), group=self.group, async_op=True)

        def fin():
            if contig is not t:
                t.copy_(contig.to(t.dtype) if t.dtype != contig.dtype else contig)

        return MPIRequest(work, fin)

    def Bcast(self, buf, root: int = 0) -> None:
        self.Ibcast(buf, root).Wait()

    # ---------------------------------------------------------------- reductions
    def _stack_async(self, src: torch.Tensor):
        """All-gather ``src`` from every rank into a [p, *src.shape] tensor (async)."""
        flat = src.reshape(-1)
        out = torch.empty(self.size * flat.numel(), dtype=src.dtype, device=src.device)
        work = _SD.all_gather_into_tensor(out, flat, group=self.group, async_op=True)
        return out.view((self.size,) + tuple(src.shape)), work

    def _fold_gathered(self, stacked: torch.Tensor, op: Op, upto: Optional[int] = None) -> torch.Tensor:
        n = stacked.shape[0] if upto is None else upto
        acc = stacked[0]
        for r in range(1, n):
            acc = op.fold(acc, stacked[r])
        return acc

    def _ipc_allreduce(self, t: torch.Tensor):
        """The one-shot xGMI all-reduce (``parallel/ipc.py``) for small device SUMs when enabled
        (``HEAT_IPC_ALLREDUCE=1``) on a node-local world communicator; None where it does not apply.
        The decision depends only on SPMD-identical facts, so every rank takes the same path."""
        from ..parallel import ipc

        if not (ipc.enabled() and t.is_cuda and self.group is None and t.is_contiguous()
                and t.dtype in (torch.float32, torch.float64, torch.int64)
                and t.numel() * t.element_size() <= ipc.max_bytes()
                and int(os.environ.get("LOCAL_WORLD_SIZE", "0")) == dist.get_world_size() == self.size):
            return None
        ar = getattr(self, "_ipc", None)
        if ar is None:
            ar = self._ipc = ipc.IpcAllreduce(self, capacity_bytes=ipc.max_bytes())
        return ar.allreduce_(t)

    def _ipc_allgather(self, moved: torch.Tensor, counts: Sequence[int]):
        """Direct W-peer xGMI all-gather (``parallel/ipc.py``) of device row blocks when IPC
        collectives are enabled on a node-local world communicator; None where it does not apply
        (same SPMD-identical conditions as ``_ipc_allreduce``, plus blocks of whole 32-bit words)."""
        from ..parallel import ipc

        row = int(np.prod(moved.shape[1:])) * moved.element_size() if moved.dim() > 1 else moved.element_size()
        if not (ipc.enabled() and moved.is_cuda and self.group is None and moved.is_contiguous()
                and row % 4 == 0 and max(counts) * row <= ipc.max_bytes()
                and int(os.environ.get("LOCAL_WORLD_SIZE", "0")) == dist.get_world_size() == self.size):
            return None
        ar = getattr(self, "_ipc", None)
        if ar is None:
            ar = self._ipc = ipc.IpcAllreduce(self, capacity_bytes=ipc.max_bytes())
        flat = ar.allgather(moved, [c * row for c in counts])
        if flat is None:
            return None
        return flat.view(moved.dtype).reshape((sum(counts),) + tuple(moved.shape[1:]))

    def _native(self):
        """The native stream-ordered RCCL communicator of this group (``HEAT_COMM_NATIVE=1``,
        device jobs of several ranks only; created collectively on first use)."""
        nc = getattr(self, "_native_comm", None)
        if nc is None:
            from ..parallel import native_comm

            nc = False
            if native_comm.enabled() and self.size > 1 and torch.cuda.is_available():
                nc = native_comm.NativeComm(self)
            self._native_comm = nc
        return nc or None

    def _reduce_tensor_async(self, t: torch.Tensor, op: Op):
        """All-reduce ``t`` in place (returns (work, finalize))."""
        if op is MPI.SUM and self._ipc_allreduce(t) is not None:
            PATH_COUNTS["allreduce:ipc"] += 1
            return None, None  # stream-ordered on the current stream: nothing to wait for
        opname = {MPI.SUM: "sum", MPI.PROD: "prod", MPI.MAX: "max", MPI.MIN: "min"}.get(op)
        if t.is_cuda and opname is not None and self._native() is not None and self._native().supports(t, opname):
            nc = self._native()
            contig = t if t.is_contiguous() else t.contiguous()
            nc.allreduce_(contig, opname)  # ordered on the current stream: nothing to wait for
            PATH_COUNTS["allreduce:native"] += 1
            if contig is not t:
                t.copy_(contig)
            return None, None
        native = op.torch_op is not None and t.dtype != torch.bool and (not t.is_complex() or op is MPI.SUM)
        if native:
            contig = _wire_dtype(t) if t.is_contiguous() else _wire_dtype(t).contiguous()
            work = _SD.all_reduce(contig, op=op.torch_op, group=self.group, async_op=True)
            PATH_COUNTS["allreduce:pg"] += 1

            def fin():
                if contig is not t:
                    t.copy_(contig.to(t.dtype) if contig.dtype != t.dtype else contig)

            return work, fin
        if op in (MPI.LAND, MPI.LOR) and op.torch_op is None:
            contig = t.to(torch.uint8).contiguous() if t.dtype == torch.bool else (t != 0).to(torch.uint8)
            rop = dist.ReduceOp.MIN if op is MPI.LAND else dist.ReduceOp.MAX
            work = _SD.all_reduce(contig, op=rop, group=self.group, async_op=True)

            def fin():
                t.copy_(contig.to(t.dtype))

            return work, fin
        # generic: all-gather the partials, fold on device (p <= 8 per node)
        src = _wire_dtype(t).contiguous()
        gathered, work = self._stack_async(src)

        def fin():
            g = gathered.to(t.dtype) if gathered.dtype != t.dtype else gathered
            t.copy_(self._fold_gathered(g, op))

        return work, fin

    def Iallreduce(self, sendbuf, recvbuf, op: Op = MPI.SUM) -> MPIRequest:
        recv = _as_tensor(recvbuf)
        if sendbuf is not MPI.IN_PLACE:
            send = _as_tensor(sendbuf)
            if send is not recv:
                recv.copy_(send.reshape(recv.shape) if send.shape != recv.shape else send)
        self._trace("Allreduce", recv)
        if self.size == 1:
            return MPIRequest()
        work, fin = self._reduce_tensor_async(recv, op)
        return MPIRequest(work, fin)

    def Allreduce(self, sendbuf, recvbuf, op: Op = MPI.SUM):
        self.Iallreduce(sendbuf, recvbuf, op).Wait()

    def Ireduce(self, sendbuf, recvbuf, op: Op = MPI.SUM, root: int = 0) -> MPIRequest:
        # the all-reduce is as cheap as a reduce on xGMI and keeps every buffer well defined
        recv = _as_tensor(recvbuf)
        if sendbuf is MPI.IN_PLACE:
            tmp = recv
        else:
            send = _as_tensor(sendbuf)
            tmp = send.clone()
        req = self.Iallreduce(MPI.IN_PLACE, tmp, op)

        def fin():
            req.Wait()
            if self.rank == root and recv is not None and tmp is not recv:
                recv.copy_(tmp.reshape(recv.shape))

        return MPIRequest(None, fin)

    def Reduce(self, sendbuf, recvbuf, op: Op = MPI.SUM, root: int = 0):
        self.Ireduce(sendbuf, recvbuf, op, root).Wait()

    def _scan(self, sendbuf, recvbuf, op: Op, exclusive: bool) -> MPIRequest:
        recv = _as_tensor(recvbuf)
        send = recv if sendbuf is MPI.IN_PLACE else _as_tensor(sendbuf)
        src = _wire_dtype(send).contiguous()
        if self.size == 1:
            if not exclusive and send is not recv:
                recv.copy_(send)
            return MPIRequest()
        gathered, work = self._stack_async(src)

        def fin():
            g = gathered.to(send.dtype) if gathered.dtype != send.dtype else gathered
            n = self.rank if exclusive else self.rank + 1
            if n == 0:
                return  # MPI leaves rank 0's Exscan receive buffer undefined; keep it untouched
            recv.copy_(self._fold_gathered(g, op, upto=n).reshape(recv.shape))

        return MPIRequest(work, fin)

    def Iexscan(self, sendbuf, recvbuf, op: Op = MPI.SUM) -> MPIRequest:
        return self._scan(sendbuf, recvbuf, op, True)

    def Exscan(self, sendbuf, recvbuf, op: Op = MPI.SUM):
        self.Iexscan(sendbuf, recvbuf, op).Wait()

    def Iscan(self, sendbuf, recvbuf, op: Op = MPI.SUM) -> MPIRequest:
        return self._scan(sendbuf, recvbuf, op, False)

    def Scan(self, sendbuf, recvbuf, op: Op = MPI.SUM):
        self.Iscan(sendbuf, recvbuf, op).Wait()

    # ---------------------------------------------------------------- all-gather
    def allgather_sizes(self, n: int) -> List[int]:
        """All-gather one integer per rank (host-side, tiny)."""
        if self.size == 1:
            return [int(n)]
        t = torch.tensor([int(n)], dtype=torch.int64, device=self._small_device())
        out = torch.empty(self.size, dtype=torch.int64, device=t.device)
        _SD.all_gather_into_tensor(out, t, group=self.group)
        return [int(x) for x in out.tolist()]

    def _small_device(self):
        b = dist.get_backend(self.group) if self.size > 1 else "gloo"
        if b == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def _allgatherv_async(self, send: torch.Tensor, axis: int, counts: Optional[Sequence[int]] = None):
        """Concatenate every rank's ``send`` along ``axis``. Returns (work, finalize -> tensor)."""
        send = _wire_dtype(send)
        moved = send.movedim(axis, 0) if axis != 0 else send
        moved = moved.contiguous()
        if counts is None:
            counts = self.allgather_sizes(moved.shape[0])
        rest = tuple(moved.shape[1:])
        got = self._ipc_allgather(moved, counts) if len(counts) else None
        path = "ipc"
        if got is None and moved.is_cuda and len(counts) and self._native() is not None \
                and moved.dtype in (torch.int8, torch.uint8, torch.bool, torch.int32, torch.int64, torch.float16,
                                    torch.float32, torch.float64, torch.bfloat16):
            got = self._native().allgatherv(moved, counts)  # grouped RCCL p2p on the current stream
            path = "native"
        if got is not None:
            PATH_COUNTS["allgatherv:" + path] += 1
            return _SD.StagedWork(None), (lambda: got.movedim(0, axis) if axis != 0 else got)
        mx = max(counts) if len(counts) else 0
        if all(c == mx for c in counts):
            padded = moved
        else:
            padded = torch.zeros((mx,) + rest, dtype=moved.dtype, device=moved.device)
            padded[: moved.shape[0]] = moved
        out = torch.empty((self.size * mx,) + rest, dtype=moved.dtype, device=moved.device)
        work = _SD.all_gather_into_tensor(out, padded, group=self.group, async_op=True)
        PATH_COUNTS["allgatherv:pg"] += 1

        def fin():
            if all(c == mx for c in counts):
                res = out
            else:
                res = torch.cat([out[r * mx: r * mx + counts[r]] for r in range(self.size)], dim=0)
            return res.movedim(0, axis) if axis != 0 else res

        return work, fin

    def reduce_scatter_tensor(self, out: torch.Tensor, inp: torch.Tensor, op: Op = None) -> torch.Tensor:
        """``out`` = this rank's 1/size block (along dim 0) of the element-wise SUM (or ``op``) of
        every rank's ``inp`` - the native stream-ordered RCCL reduce-scatter under
        ``HEAT_COMM_NATIVE=1``, else torch's (host-staged for a gloo group)."""
        op = MPI.SUM if op is None else op
        self._trace("Reduce_scatter", inp)
        if self.size == 1:
            return out.copy_(inp)
        opname = {MPI.SUM: "sum", MPI.PROD: "prod", MPI.MAX: "max", MPI.MIN: "min"}.get(op)
        nc = self._native() if inp.is_cuda else None
        if nc is not None and opname is not None and nc.supports(inp, opname) and inp.is_contiguous() \
                and out.is_contiguous():
            PATH_COUNTS["reduce_scatter:native"] += 1
            return nc.reduce_scatter(inp, out, opname)
        PATH_COUNTS["reduce_scatter:pg"] += 1
        _SD.reduce_scatter_tensor(out, inp, op=op.torch_op, group=self.group)
        return out

    def allgather_tensor(self, t: torch.Tensor, axis: int = 0, counts: Optional[Sequence[int]] = None) -> torch.Tensor:
        """Return the concatenation of all ranks' tensors along ``axis`` (sizes may differ)."""
        if self.size == 1:
            return t
        dtype = t.dtype
        work, fin = self._allgatherv_async(t, axis, counts)
        work.wait()
        res = fin()
        return res.to(dtype) if res.dtype != dtype else res

    def _unpack_v(self, buf):
        counts = displs = None
        if isinstance(buf, tuple):
            if len(buf) == 3:
                buf, counts, displs = buf
            elif len(buf) == 2:
                buf, counts = buf[0], buf[1]
                if isinstance(counts, (tuple, list)) and len(counts) == 2 and isinstance(counts[0], (tuple, list)):
                    counts, displs = counts
            else:
                buf = buf[0]
        return _as_tensor(buf), counts, displs

    def Iallgatherv(self, sendbuf, recvbuf, recv_axis: int = 0) -> MPIRequest:
        recv, counts, displs = self._unpack_v(recvbuf)
        if sendbuf is MPI.IN_PLACE:
            if counts is None:
                counts = self.counts_displs_shape(recv.shape, recv_axis)[0]
            off = sum(counts[: self.rank])
            send = recv.narrow(recv_axis, off, counts[self.rank]).clone()
        else:
            send, _, _ = self._unpack_v(sendbuf)
        self._trace("Allgatherv", send)
        if self.size == 1:
            if send.data_ptr() != recv.data_ptr():
                recv.copy_(send.reshape(recv.shape))
            return MPIRequest()
        if counts is not None:
            counts = [int(c) for c in (counts.tolist() if isinstance(counts, torch.Tensor) else counts)]
        work, fin = self._allgatherv_async(send, recv_axis, counts)

        def fin2():
            res = fin()
            recv.copy_(res.to(recv.dtype).reshape(recv.shape))

        return MPIRequest(work, fin2)

    def Allgatherv(self, sendbuf, recvbuf, recv_axis: int = 0):
        self.Iallgatherv(sendbuf, recvbuf, recv_axis).Wait()

    def Iallgather(self, sendbuf, recvbuf, recv_axis: int = 0) -> MPIRequest:
        recv, _, _ = self._unpack_v(recvbuf)
        if sendbuf is MPI.IN_PLACE:
            return self.Iallgatherv(MPI.IN_PLACE, recvbuf, recv_axis)
        send, _, _ = self._unpack_v(sendbuf)
        if self.size == 1:
            recv.copy_(send.reshape(recv.shape))
            return MPIRequest()
        if send.dim() == 0:
            send = send.reshape(1)
        n = send.shape[recv_axis] if send.dim() > recv_axis else 1
        work, fin = self._allgatherv_async(send, recv_axis, [n] * self.size)

        def fin2():
            res = fin()
            recv.copy_(res.to(recv.dtype).reshape(recv.shape))

        return MPIRequest(work, fin2)

    def Allgather(self, sendbuf, recvbuf, recv_axis: int = 0):
        self.Iallgather(sendbuf, recvbuf, recv_axis).Wait()

    # ---------------------------------------------------------------- gather / scatter
    def Igatherv(self, sendbuf, recvbuf, root: int = 0, axis: int = 0, recv_axis: int = None) -> MPIRequest:
        """Concatenation of every rank's block along ``axis`` on ``root`` only: one size exchange
        and one personalised exchange in which only ``root`` receives (no all-gather)."""
        axis = axis if recv_axis is None else recv_axis
        send, _, _ = self._unpack_v(sendbuf)
        recv = self._unpack_v(recvbuf)[0] if recvbuf is not None else None
        if self.size == 1:
            if recv is not None:
                recv.copy_(send.reshape(recv.shape))
            return MPIRequest()
        if send.dim() == 0:
            send = send.reshape(1)
        self._trace("Gatherv", send)
        counts = self.allgather_sizes(send.shape[axis])
        blocks = [send if r == root else send.narrow(axis, 0, 0) for r in range(self.size)]
        if self.rank == root:
            shapes = []
            for r in range(self.size):
                s_ = list(send.shape)
                s_[axis] = counts[r]
                shapes.append(tuple(s_))
        else:
            shapes = [tuple(send.narrow(axis, 0, 0).shape)] * self.size
        work, fin = self._exchange_async(blocks, shapes)

        def done():
            out = fin()
            if self.rank == root and recv is not None:
                recv.copy_(torch.cat(out, dim=axis).to(recv.dtype).reshape(recv.shape))

        return MPIRequest(work, done)

    def Gatherv(self, sendbuf, recvbuf, root: int = 0, axis: int = 0, recv_axis: int = None):
        self.Igatherv(sendbuf, recvbuf, root, axis, recv_axis).Wait()

    Igather = Igatherv
    Gather = Gatherv

    def Iscatterv(self, sendbuf, recvbuf, root: int = 0, axis: int = 0) -> MPIRequest:
        recv, _, _ = self._unpack_v(recvbuf)
        if self.size == 1:
            send, _, _ = self._unpack_v(sendbuf)
            recv.copy_(send.reshape(recv.shape))
            return MPIRequest()
        # root broadcasts nothing but its chunks: one all_to_all where only root sends
        counts = self.allgather_sizes(recv.shape[axis])
        blocks = []
        if self.rank == root:
            send, scounts, sdispls = self._unpack_v(sendbuf)
            if scounts is not None:
                counts = [int(c) for c in scounts]
            off = 0
            for r in range(self.size):
                blocks.append(send.narrow(axis, off, counts[r]))
                off += counts[r]
        else:
            blocks = [recv.new_empty((0,)) for _ in range(self.size)]
        recv_shapes = [tuple(recv.shape) if r == root else (0,) for r in range(self.size)]
        work, fin = self._exchange_async(blocks, recv_shapes)

        def done():
            recv.copy_(fin()[root].reshape(recv.shape))

        return MPIRequest(work, done)

    def Scatterv(self, sendbuf, recvbuf, root: int = 0, axis: int = 0):
        self.Iscatterv(sendbuf, recvbuf, root, axis).Wait()

    Iscatter = Iscatterv
    Scatter = Scatterv

    # ---------------------------------------------------------------- all-to-all
    def exchange(self, send_blocks: List[torch.Tensor], recv_shapes: List[Tuple[int, ...]]) -> List[torch.Tensor]:
        """Personalised exchange: ``send_blocks[r]`` goes to rank r, the block from rank r has
        shape ``recv_shapes[r]``. One packed ``all_to_all_single`` (RCCL grouped p2p over xGMI)."""
        work, fin = self._exchange_async(send_blocks, recv_shapes)
        if work is not None:
            work.wait()
        return fin()

    def _exchange_async(self, send_blocks, recv_shapes):
        """Start :meth:`exchange`; returns (work or None, finalize -> list of received blocks)."""
        if self.size == 1:
            blk = send_blocks[0].reshape(recv_shapes[0])
            return None, lambda: [blk]
        ref = next((b for b in send_blocks if b is not None), None)
        dtype, device = ref.dtype, ref.device
        wire = _WIRE.get(dtype, dtype)
        in_sizes = [int(b.numel()) for b in send_blocks]
        out_sizes = [int(np.prod(s)) if len(s) else 1 for s in recv_shapes]
        flat_in = torch.cat([b.reshape(-1).to(wire) for b in send_blocks]) if sum(in_sizes) else \
            torch.empty(0, dtype=wire, device=device)
        flat_out = torch.empty(sum(out_sizes), dtype=wire, device=device)
        if flat_in.is_complex():
            fi, fo = torch.view_as_real(flat_in).reshape(-1), torch.view_as_real(flat_out).reshape(-1)
            work = _SD.all_to_all_single(fo, fi, [2 * s for s in out_sizes], [2 * s for s in in_sizes],
                                          group=self.group, async_op=True)
        else:
            work = _SD.all_to_all_single(flat_out, flat_in, out_sizes, in_sizes, group=self.group, async_op=True)

        def fin():
            res, off = [], 0
            for s, n in zip(recv_shapes, out_sizes):
                res.append(flat_out[off: off + n].reshape(s).to(dtype))
                off += n
            return res

        return work, fin

    def exchange_axis_async(self, send: torch.Tensor, send_axis: int, scounts, recv_shape, recv_axis: int, rcounts):
        """Personalised exchange of the blocks ``send.narrow(send_axis, ., scounts[q])`` (to rank q);
        the block from rank r lands in ``recv.narrow(recv_axis, ., rcounts[r])`` of a new tensor of
        ``recv_shape``. The send blocks are packed into one buffer and the receive buffer unpacked
        in one pass each (native ``pack.hip`` kernels on the GPU), the wire is the raw bytes (any
        dtype, one ``all_to_all_single``). Returns (work or None, finalize -> recv tensor)."""
        from ..ops import kernels as _k

        recv_shape = tuple(int(x) for x in recv_shape)
        if self.size == 1:
            out = send.reshape(recv_shape) if tuple(send.shape) == recv_shape else send
            return None, lambda: out
        packed = _k.pack_blocks(send, send_axis, scounts)
        in_b, out_b = exchange_axis_bytes(tuple(send.shape), send_axis, scounts, recv_shape, recv_axis, rcounts,
                                          send.element_size())
        flat_out = torch.empty(int(np.prod(recv_shape)) if recv_shape else 1, dtype=send.dtype, device=send.device)
        src_b = packed.contiguous().view(torch.uint8) if packed.numel() else torch.empty(0, dtype=torch.uint8,
                                                                                           device=send.device)
        dst_b = flat_out.view(torch.uint8) if flat_out.numel() else torch.empty(0, dtype=torch.uint8,
                                                                                device=send.device)
        if send.is_cuda and self._native() is not None:
            self._native().alltoallv_bytes(src_b, in_b, dst_b, out_b)  # on the current stream
            return None, lambda: _k.unpack_blocks(flat_out, recv_shape, recv_axis, rcounts)
        work = _SD.all_to_all_single(dst_b, src_b, out_b, in_b, group=self.group, async_op=True)
        return work, lambda: _k.unpack_blocks(flat_out, recv_shape, recv_axis, rcounts)

    def exchange_axis(self, send, send_axis, scounts, recv_shape, recv_axis, rcounts) -> torch.Tensor:
        """Blocking :meth:`exchange_axis_async`."""
        self._trace("Alltoallv", send)
        work, fin = self.exchange_axis_async(send, send_axis, scounts, recv_shape, recv_axis, rcounts)
        if work is not None:
            work.wait()
        return fin()

    def _alltoall_impl(self, sendbuf, recvbuf, send_axis, recv_axis) -> MPIRequest:
        send, scounts, _ = self._unpack_v(sendbuf)
        recv, rcounts, _ = self._unpack_v(recvbuf)
        if recv_axis is None:
            recv_axis = send_axis
        if scounts is None:
            scounts = self.counts_displs_shape(send.shape, send_axis)[0]
        if rcounts is None:
            rcounts = self.counts_displs_shape(recv.shape, recv_axis)[0]
        scounts = [int(c) for c in scounts]
        rcounts = [int(c) for c in rcounts]
        self._trace("Alltoallv", send)
        work, fin = self.exchange_axis_async(send, send_axis, scounts, tuple(recv.shape), recv_axis, rcounts)

        def done():
            res = fin()
            if res.data_ptr() != recv.data_ptr():
                recv.copy_(res.reshape(recv.shape))

        return MPIRequest(work, done)

    def Ialltoallv(self, sendbuf, recvbuf, send_axis: int = 0, recv_axis: int = None) -> MPIRequest:
        return self._alltoall_impl(sendbuf, recvbuf, send_axis, recv_axis)

    def Alltoallv(self, sendbuf, recvbuf, send_axis: int = 0, recv_axis: int = None):
        self._alltoall_impl(sendbuf, recvbuf, send_axis, recv_axis).Wait()

    Ialltoall = Ialltoallv
    Alltoall = Alltoallv

    # ---------------------------------------------------------------- point to point
    def _tag(self, tag):
        # RCCL has no tags: ordering per (src, dst) pair is FIFO; gloo honours them
        return int(tag) if tag is not None and tag >= 0 else 0

    def _mailbox(self):
        """Messages a rank sends to itself (MPI allows it; torch.distributed has no self-send):
        FIFO per tag, matched by the receive when it is waited on."""
        box = getattr(self, "_self_box", None)
        if box is None:
            import collections

            box = self._self_box = collections.defaultdict(collections.deque)
        return box

    def _take_self(self, tag):
        box = self._mailbox()
        if tag is None or tag == MPI.ANY_TAG:
            tag = next((k for k, q in box.items() if q), None)
        if tag is None or not box[self._tag(tag)]:
            raise RuntimeError("receive from self without a matching send posted before the wait")
        return box[self._tag(tag)].popleft()

    def Isend(self, buf, dest: int, tag: int = 0) -> MPIRequest:
        t = _as_tensor(buf)
        if not isinstance(t, torch.Tensor):
            return self.isend(buf, dest, tag)
        if dest == self.rank:
            self._mailbox()[self._tag(tag)].append(t.clone())
            return MPIRequest()
        src = _wire_dtype(t).contiguous()
        work = _SD.isend(src, dst=self._g(dest), group=self.group, tag=self._tag(tag))
        return MPIRequest(work, result=src)

    def Send(self, buf, dest: int, tag: int = 0):
        self.Isend(buf, dest, tag).Wait()

    Ssend = Rsend = Bsend = Send
    Issend = Irsend = Ibsend = Isend

    def Irecv(self, buf, source: int = MPI.ANY_SOURCE, tag: int = MPI.ANY_TAG) -> MPIRequest:
        t = _as_tensor(buf)
        if isinstance(buf, tuple):
            t = _as_tensor(buf[0])
        dst = t if (t.is_contiguous() and t.dtype not in _WIRE) else torch.empty_like(_wire_dtype(t)).contiguous()
        if source == self.rank:
            return MPIRequest(None, lambda: t.copy_(self._take_self(tag).reshape(t.shape).to(t.dtype)))
        if source == MPI.ANY_SOURCE:
            raise NotImplementedError("ANY_SOURCE receives are not supported over RCCL; name the peer")
        work = _SD.irecv(dst, src=self._g(source), group=self.group, tag=self._tag(tag))

        def fin():
            if dst is not t:
                t.copy_(dst.to(t.dtype))

        return MPIRequest(work, fin)

    def Recv(self, buf, source: int = MPI.ANY_SOURCE, tag: int = MPI.ANY_TAG, status=None):
        self.Irecv(buf, source, tag).Wait()

    def sendrecv_tensor(self, send: Optional[torch.Tensor], dest: Optional[int],
                        recv_shape, source: Optional[int], dtype=None, device=None) -> Optional[torch.Tensor]:
        """Simultaneous send to ``dest`` and receive from ``source`` (either may be None)."""
        ops = []
        out = None
        if send is not None and dest is not None:
            s = _wire_dtype(send).contiguous()
            ops.append(dist.P2POp(dist.isend, s, self._g(dest), self.group))
            dtype = dtype or send.dtype
            device = device or send.device
        if source is not None:
            dtype = dtype or torch.float32
            wire = _WIRE.get(dtype, dtype)
            out = torch.empty(tuple(recv_shape), dtype=wire, device=device)
            ops.append(dist.P2POp(dist.irecv, out, self._g(source), self.group))
        if ops:
            for w in _SD.batch_isend_irecv(ops):
                w.wait()
        if out is not None and out.dtype != dtype:
            out = out.to(dtype)
        return out

    # ---------------------------------------------------------------- pickled object ops
    def _obj_device(self):
        return self._small_device()

    def bcast(self, obj: Any, root: int = 0) -> Any:
        if self.size == 1:
            return obj
        lst = [obj if self.rank == root else None]
        dist.broadcast_object_list(lst, src=self._g(root), group=self.group)
        return lst[0]

    def allgather(self, obj: Any) -> List[Any]:
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def gather(self, obj: Any, root: int = 0) -> Optional[List[Any]]:
        res = self.allgather(obj)
        return res if self.rank == root else None

    def scatter(self, objs: Optional[Sequence[Any]], root: int = 0) -> Any:
        if self.size == 1:
            return objs[0]
        return self.bcast(list(objs) if self.rank == root else None, root)[self.rank]

    def allreduce(self, obj: Any, op: Op = MPI.SUM) -> Any:
        vals = self.allgather(obj)
        acc = vals[0]
        for v in vals[1:]:
            if op is MPI.SUM:
                acc = acc + v
            elif op is MPI.PROD:
                acc = acc * v
            elif op is MPI.MAX:
                acc = max(acc, v)
            elif op is MPI.MIN:
                acc = min(acc, v)
            elif op is MPI.LAND:
                acc = bool(acc) and bool(v)
            elif op is MPI.LOR:
                acc = bool(acc) or bool(v)
            else:
                acc = op.fold(acc, v)
        return acc

    def alltoall(self, objs: Sequence[Any]) -> List[Any]:
        gathered = self.allgather(list(objs))
        return [gathered[r][self.rank] for r in range(self.size)]

    def _obj_to_tensor(self, obj):
        data = pickle.dumps(obj)
        dev = self._obj_device()
        payload = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        size = torch.tensor([payload.numel()], dtype=torch.int64, device=dev)
        return size, payload

    def isend(self, obj: Any, dest: int, tag: int = 0) -> MPIRequest:
        if dest == self.rank:
            self._mailbox()[self._tag(tag)].append(pickle.dumps(obj))
            return MPIRequest()
        size, payload = self._obj_to_tensor(obj)
        w1 = _SD.isend(size, dst=self._g(dest), group=self.group, tag=self._tag(tag))
        w2 = _SD.isend(payload, dst=self._g(dest), group=self.group, tag=self._tag(tag))
        return MPIRequest([w1, w2], result=(size, payload))

    def send(self, obj: Any, dest: int, tag: int = 0):
        self.isend(obj, dest, tag).Wait()

    def recv(self, buf=None, source: int = 0, tag: int = 0, status=None) -> Any:
        if source == self.rank:
            return pickle.loads(self._take_self(tag))
        dev = self._obj_device()
        size = torch.empty(1, dtype=torch.int64, device=dev)
        _SD.recv(size, src=self._g(source), group=self.group, tag=self._tag(tag))
        payload = torch.empty(int(size.item()), dtype=torch.uint8, device=dev)
        _SD.recv(payload, src=self._g(source), group=self.group, tag=self._tag(tag))
        return pickle.loads(payload.cpu().numpy().tobytes())

    def irecv(self, buf=None, source: int = 0, tag: int = 0) -> MPIRequest:
        return MPIRequest(None, lambda: self.recv(buf, source, tag))

    def sendrecv(self, sendobj: Any, dest: int, sendtag: int = 0, recvbuf=None, source: int = None,
                 recvtag: int = None, status=None) -> Any:
        source = dest if source is None else source
        req = self.isend(sendobj, dest, sendtag)
        obj = self.recv(recvbuf, source, sendtag if recvtag is None else recvtag)
        req.Wait()
        return obj

    # ---------------------------------------------------------------- sub-communicators
    def Split(self, color: int = 0, key: int = 0) -> "MPICommunication":
        """Collective: split into sub-communicators by ``color``, ordered by ``key``."""
        if self.size == 1:
            return MPICommunication(_self_only=True)
        entries = self.allgather((color, key, self.rank, self._g(self.rank)))
        colors = sorted(set(e[0] for e in entries if e[0] != MPI.UNDEFINED))
        mine = None
        for c in colors:
            members = sorted([e for e in entries if e[0] == c], key=lambda e: (e[1], e[2]))
            granks = [e[3] for e in members]
            grp = dist.new_group(ranks=granks)
            if c == color:
                mine = MPICommunication(grp, granks) if len(granks) > 1 else MPICommunication(_self_only=True)
        return mine

    def Create_group(self, ranks: Sequence[int]) -> Optional["MPICommunication"]:
        """Collective: communicator over the given (group-relative) ranks."""
        granks = [self._g(r) for r in ranks]
        if self.size == 1:
            return MPICommunication(_self_only=True)
        grp = dist.new_group(ranks=granks)
        if self._g(self.rank) in granks:
            return MPICommunication(grp, granks) if len(granks) > 1 else MPICommunication(_self_only=True)
        return None

    Create = Create_group

    def Dup(self) -> "MPICommunication":
        return self

    def Free(self):
        pass

    def Abort(self, errorcode: int = 1):
        os._exit(errorcode)

    def Get_group(self):
        return self._ranks

    @property
    def ranks(self) -> List[int]:
        return list(self._ranks)


# alias with a name that says what it is
TorchCommunication = MPICommunication

MPI_WORLD = MPICommunication()
MPI_SELF = MPICommunication(_self_only=True)

# the communicator used by default
__default_comm = MPI_WORLD


def get_comm() -> Communication:
    """The process-wide default communicator (COMM_WORLD unless ``use_comm`` changed it)."""
    return __default_comm


def sanitize_comm(comm: Optional[Communication]) -> Communication:
    """``comm`` if it is a Communication, the default communicator for None; TypeError otherwise."""
    if comm is None:
        return get_comm()
    if isinstance(comm, Communication):
        return comm
    raise TypeError("Unknown communication, must be instance of {}".format(Communication))


def use_comm(comm: Communication = None):
    """Make ``comm`` (or COMM_WORLD for None) the default communicator of new arrays."""
    global __default_comm
    __default_comm = sanitize_comm(comm)
