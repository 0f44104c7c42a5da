"""
Intra-node collectives over hipIpc-mapped peer buffers (kernels in
``ops/csrc/ipc_allreduce.hip``): one-shot all-reduce, two-shot (reduce-scatter + all-gather)
all-reduce above ``HEAT_IPC_TWOSHOT_BYTES``, and a direct W-peer all-gather.

For the small payloads the framework reduces once per algorithmic step (k-means' packed k*f + k
sums, moment triples, arg-reduction packs, metadata maps) one kernel does the whole collective:
every rank copies its input into an IPC-exported slot, raises per-block flags in every peer's
signal buffer and sums the peers' slots straight over xGMI - one launch, no RCCL channel set-up,
bitwise identical results on every rank (fixed rank-order summation).

``IpcAllreduce(comm)`` is collective to construct (handle exchange through the host object
all-gather) and is used by :class:`heat_amd.core.communication.MPICommunication` for SUM
all-reduces of device float32/float64/int64 tensors up to ``HEAT_IPC_MAX_BYTES`` when
``HEAT_IPC_ALLREDUCE=1`` and every rank of the communicator is on this node.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

_DTYPES = {torch.float32: 0, torch.float64: 1, torch.int64: 2}


def _lib():
    from .. import ops

    L = ops.lib()
    c_void_p, c_int, c_int64, c_uint = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint
    for name, res, args in (
            ("ha_ipc_handle_size", c_int, []),
            ("ha_ipc_max_ranks", c_int, []),
            ("ha_ipc_max_blocks", c_int, []),
            ("ha_ipc_signal_bytes", c_int64, []),
            ("ha_ipc_alloc", c_int, [c_int64, c_int, ctypes.POINTER(c_void_p), c_void_p]),
            ("ha_ipc_free", c_int, [c_void_p]),
            ("ha_ipc_open", c_int, [c_void_p, ctypes.POINTER(c_void_p)]),
            ("ha_ipc_close", c_int, [c_void_p]),
            ("ha_ipc_allreduce", c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_int, c_void_p,
                                         c_int64, c_int, c_int64, c_uint, c_int, c_int64, c_int, c_void_p]),
            ("ha_ipc_allgather", c_int, [ctypes.POINTER(c_void_p), ctypes.POINTER(c_void_p), c_int, c_int, c_void_p,
                                         c_void_p, ctypes.POINTER(c_int64), ctypes.POINTER(c_int64), c_int64, c_uint,
                                         c_int, c_int64, c_void_p]),
            ("ha_ipc_error", c_int, [c_void_p, c_int]),
            ("ha_ipc_error_async", c_int, [c_void_p, c_void_p, c_void_p])):
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    return L


class IpcTimeoutError(RuntimeError):
    """A peer missed an IPC barrier: the affected output was poisoned (NaN) and the communicator
    cannot be used again (slot reuse is only safe while every barrier completes)."""


def _check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError("IPC all-reduce: {} failed with status {}".format(what, rc))


class IpcAllreduce:
    """SUM all-reduce (one-shot / two-shot) and all-gather among the ranks of ``comm`` (all on
    this node, one GPU each, or several ranks sharing a GPU in tests). ``capacity_bytes``: the
    largest all-reduce payload / per-rank all-gather block."""

    def __init__(self, comm, capacity_bytes: int = 4 << 20, blocks: int = 32, timeout_spins: int = 4_000_000):
        L = _lib()
        self.comm = comm
        self.world, self.rank = comm.size, comm.rank
        if not 2 <= self.world <= L.ha_ipc_max_ranks():
            raise ValueError("IPC all-reduce supports 2..{} ranks, got {}".format(L.ha_ipc_max_ranks(), self.world))
        self.capacity = int(capacity_bytes)
        self.blocks = max(1, min(int(blocks), L.ha_ipc_max_blocks()))
        self.spins = int(timeout_spins)
        self.two_shot_bytes = two_shot_bytes()
        self.epoch = 0
        self.device = torch.device("cuda", torch.cuda.current_device())
        hs = L.ha_ipc_handle_size()
        self._own = []
        handles = []
        for nbytes, signal in ((2 * self.capacity, 0), (L.ha_ipc_signal_bytes(), 1)):
            ptr, h = ctypes.c_void_p(), ctypes.create_string_buffer(hs)
            _check(L.ha_ipc_alloc(nbytes, signal, ctypes.byref(ptr), h), "alloc")
            self._own.append(ptr.value)
            handles.append(h.raw)
        allh = comm.allgather(handles)
        self._opened = []
        data, sig = [], []
        for r, (hd, hsig) in enumerate(allh):
            if r == self.rank:
                data.append(self._own[0])
                sig.append(self._own[1])
                continue
            ptrs = []
            for h in (hd, hsig):
                p = ctypes.c_void_p()
                _check(L.ha_ipc_open(ctypes.create_string_buffer(h, hs), ctypes.byref(p)), "open peer handle")
                self._opened.append(p.value)
                ptrs.append(p.value)
            data.append(ptrs[0])
            sig.append(ptrs[1])
        arr = ctypes.c_void_p * self.world
        self._data = arr(*data)
        self._sig = arr(*sig)
        self._L = L
        # error word of every call, copied behind it on the stream into pinned host memory; the
        # next call (or check()) reads it once the copy's event has completed
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._err_event = None
        self._poisoned = False
        comm.Barrier()

    def supports(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype in _DTYPES and t.is_contiguous()
                and t.numel() * t.element_size() <= self.capacity)

    def _poll(self, wait: bool = False):
        """Raise if an earlier call of this rank timed out (reads the pinned copy of the error
        word once the copy behind that call has landed; ``wait`` blocks for it)."""
        if self._poisoned:
            raise IpcTimeoutError("IPC all-reduce disabled after an earlier barrier timeout")
        ev = self._err_event
        if ev is None:
            return
        if wait:
            ev.synchronize()
        elif not ev.query():
            return
        if int(self._err_host[0]) != 0:
            self._poisoned = True
            raise IpcTimeoutError("an IPC all-reduce barrier timed out on rank {}: its result was "
                                  "poisoned with NaN".format(self.rank))

    def check(self):
        """Block until every issued call has finished and raise if any of them timed out."""
        self._poll(wait=True)

    def _after(self, stream):
        _check(self._L.ha_ipc_error_async(ctypes.c_void_p(self._own[1]), ctypes.c_void_p(self._err_host.data_ptr()),
                                          ctypes.c_void_p(stream.cuda_stream)), "error copy")
        if self._err_event is None:
            self._err_event = torch.cuda.Event()
        self._err_event.record(stream)

    def allgather(self, t: torch.Tensor, counts_bytes) -> Optional[torch.Tensor]:
        """Concatenation of every rank's contiguous device tensor ``t`` (rank q holds
        ``counts_bytes[q]`` bytes) as a flat uint8 tensor on the current stream: every rank pulls
        its W-1 peers' blocks directly from their slots. None when a block is not a multiple of 4
        bytes or exceeds the slot."""
        counts_bytes = [int(c) for c in counts_bytes]
        if any(c % 4 or c > self.capacity for c in counts_bytes) or not t.is_contiguous() or not t.is_cuda:
            return None
        if sum(counts_bytes) == 0:
            # nothing to move and no kernel: the epoch must not advance, since the two-slot reuse
            # argument needs a barrier between consecutive epochs
            return torch.empty(0, dtype=torch.uint8, device=t.device)
        self._poll()
        self.epoch += 1
        words = [c // 4 for c in counts_bytes]
        displ = [0] * self.world
        for q in range(1, self.world):
            displ[q] = displ[q - 1] + words[q - 1]
        out = torch.empty(sum(counts_bytes), dtype=torch.uint8, device=t.device)
        arr = ctypes.c_int64 * self.world
        stream = torch.cuda.current_stream(t.device)
        rc = self._L.ha_ipc_allgather(self._data, self._sig, self.world, self.rank, ctypes.c_void_p(t.data_ptr()),
                                      ctypes.c_void_p(out.data_ptr()), arr(*words), arr(*displ), self.capacity // 4,
                                      self.epoch & 0xFFFFFFFF, self.blocks, self.spins,
                                      ctypes.c_void_p(stream.cuda_stream))
        _check(rc, "all-gather launch")
        self._after(stream)
        return out

    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM of ``t`` over the ranks, ordered on the current stream. Raises
        :class:`IpcTimeoutError` when an EARLIER call timed out (this rank's view); a timed-out
        call's own output is NaN-poisoned, so a silent wrong sum is impossible either way."""
        if not self.supports(t):
            raise ValueError("tensor not supported by the IPC all-reduce")
        if t.numel() == 0:
            return t  # no kernel launches for an empty payload: keep the epoch (see allgather)
        self._poll()
        self.epoch += 1
        es = t.element_size()
        two_shot = int(t.numel() * es > self.two_shot_bytes)
        stream = torch.cuda.current_stream(t.device)
        rc = self._L.ha_ipc_allreduce(self._data, self._sig, self.world, self.rank, ctypes.c_void_p(t.data_ptr()),
                                      t.numel(), _DTYPES[t.dtype], self.capacity // es, self.epoch & 0xFFFFFFFF,
                                      self.blocks, self.spins, two_shot, ctypes.c_void_p(stream.cuda_stream))
        _check(rc, "launch")
        self._after(stream)
        return t

    def error(self, clear: bool = False) -> int:
        """1 if a barrier of an earlier call timed out on this rank (synchronises the device)."""
        return self._L.ha_ipc_error(ctypes.c_void_p(self._own[1]), int(clear))

    def close(self):
        if self._L is None:
            return
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self._L.ha_ipc_close(ctypes.c_void_p(p))
        for p in self._own:
            self._L.ha_ipc_free(ctypes.c_void_p(p))
        self._opened, self._own, self._L = [], [], None


def enabled() -> bool:
    return os.environ.get("HEAT_IPC_ALLREDUCE", "0") == "1"


def max_bytes() -> int:
    return int(os.environ.get("HEAT_IPC_MAX_BYTES", str(16 << 20)))


def two_shot_bytes() -> int:
    """Payload above which the all-reduce runs two-shot (each rank moves 2(W-1)/W of the data
    instead of (W-1)x)."""
    return int(os.environ.get("HEAT_IPC_TWOSHOT_BYTES", str(256 << 10)))


def node_local(comm) -> bool:
    """True if every rank of ``comm`` runs on this node (one launcher, LOCAL_WORLD_SIZE >= size)."""
    lws = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    return comm.size <= lws
