"""
Native stream-ordered RCCL communicator (``ops/csrc/comm.hip``).

``NativeComm(comm)`` creates an RCCL communicator over the ranks of a heat communicator (the
unique id travels over the existing process group) on the RCCL instance torch already loaded.
Collectives run on the CALLER's current stream - ordered with the surrounding kernels, no
ProcessGroupNCCL side-stream events, capturable in a HIP graph - and return immediately.
``HEAT_COMM_NATIVE=1`` routes device SUM/MAX/MIN/PROD all-reduces, all-gathers (also of unequal
blocks: a grouped send/receive, no padding), reduce-scatters and the byte exchanges of
``exchange_axis`` through it; the default stays torch's ProcessGroupNCCL. An
asynchronous RCCL error (peer failure) is polled with :meth:`check` (the heat watchdog calls it on
every synchronising wait).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np
import torch

__all__ = ["NativeComm", "enabled", "rccl_path", "allgatherv_plan", "alltoallv_plan", "simulate_alltoallv"]

# ncclDataType_t / ncclRedOp_t codes
_DT = {torch.int8: 0, torch.uint8: 1, torch.bool: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6,
       torch.float32: 7, torch.float64: 8, torch.bfloat16: 9}
_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3}


# ------------------------------------------------------------------ byte plans (pure, CPU-testable)
def allgatherv_plan(counts: Sequence[int], rank: int, row_bytes: int):
    """Arguments of ``ha_comm_alltoallv`` for an all-gather of unequal row blocks: this rank sends
    its whole block (``counts[rank]`` rows, offset 0) to every peer and receives rank q's block at
    the byte offset of q's rows in the concatenation. Returns int64 arrays (sb, so, rb, ro)."""
    size = len(counts)
    own = int(counts[rank]) * int(row_bytes)
    sb = np.full(size, own, dtype=np.int64)
    so = np.zeros(size, dtype=np.int64)
    rb = np.asarray([int(c) * int(row_bytes) for c in counts], dtype=np.int64)
    ro = np.concatenate([[0], np.cumsum(rb)[:-1]]).astype(np.int64) if size else np.zeros(0, np.int64)
    return sb, so, rb, ro


def alltoallv_plan(send_bytes: Sequence[int], recv_bytes: Sequence[int]):
    """Arguments of ``ha_comm_alltoallv`` for blocks stored back to back in rank order on both
    sides. Returns int64 arrays (sb, so, rb, ro)."""
    sb = np.asarray(send_bytes, dtype=np.int64)
    rb = np.asarray(recv_bytes, dtype=np.int64)
    so = np.concatenate([[0], np.cumsum(sb)[:-1]]).astype(np.int64) if sb.size else np.zeros(0, np.int64)
    ro = np.concatenate([[0], np.cumsum(rb)[:-1]]).astype(np.int64) if rb.size else np.zeros(0, np.int64)
    return sb, so, rb, ro


def simulate_alltoallv(sends, plans, recv_sizes):
    """Host model of ``ha_comm_alltoallv`` run by every rank at once (``ops/csrc/comm.hip``):
    rank r's ``sends[r]`` (uint8 array) and ``plans[r]`` = (sb, so, rb, ro); returns every rank's
    receive buffer (``recv_sizes[r]`` bytes). Raises where the real exchange would fail or hang: a
    local block whose send and receive sizes differ (HA_BAD_ARG), or a send of rank r to q whose
    size differs from the receive q posted for r (mismatched RCCL p2p)."""
    size = len(sends)
    out = [np.zeros(int(n), dtype=np.uint8) for n in recv_sizes]
    for r in range(size):
        sb, so, rb, ro = plans[r]
        if sb[r] != rb[r]:
            raise ValueError("rank {}: local block sends {} bytes, receives {}".format(r, sb[r], rb[r]))
        for q in range(size):
            qsb, qso, qrb, qro = plans[q]
            if qsb[r] != rb[q]:
                raise ValueError("rank {} expects {} bytes from {}, which sends {}".format(r, rb[q], q, qsb[r]))
            if rb[q] < 0 or ro[q] + rb[q] > out[r].size or qso[r] + qsb[r] > sends[q].size:
                raise ValueError("rank {}: block from {} out of bounds".format(r, q))
            out[r][ro[q]: ro[q] + rb[q]] = sends[q][qso[r]: qso[r] + qsb[r]]
    return out


def enabled() -> bool:
    return os.environ.get("HEAT_COMM_NATIVE", "0") == "1"


def rccl_path() -> Optional[str]:
    """Path of the RCCL library mapped into this process (torch's bundled copy), else the ROCm one."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1]
                if os.path.basename(p).startswith("librccl.so"):
                    return p
    except OSError:
        pass
    for cand in ("/opt/rocm/lib/librccl.so.1", "/opt/rocm/lib/librccl.so"):
        if os.path.exists(cand):
            return cand
    return None


class NativeComm:
    """An RCCL communicator spanning ``comm``'s ranks (collective constructor)."""

    def __init__(self, comm):
        from ..ops import check, lib

        self.L = lib()
        path = rccl_path()
        if path is None:
            raise RuntimeError("no RCCL library found")
        check(self.L.ha_comm_load(path.encode()), "ha_comm_load")
        self.size, self.rank = comm.size, comm.rank
        uid = ctypes.create_string_buffer(128)
        if self.rank == 0:
            check(self.L.ha_comm_unique_id(uid), "ha_comm_unique_id")
        raw = comm.bcast(bytes(uid.raw), root=0) if self.size > 1 else bytes(uid.raw)
        uid = ctypes.create_string_buffer(raw, 128)
        handle = ctypes.c_void_p()
        check(self.L.ha_comm_init(uid, self.size, self.rank, ctypes.byref(handle)), "ha_comm_init")
        self.handle = handle

    # ------------------------------------------------------------------ collectives
    @staticmethod
    def _stream(t: torch.Tensor):
        return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)

    def supports(self, t: torch.Tensor, op: Optional[str] = None) -> bool:
        return t.is_cuda and t.dtype in _DT and (op is None or (op in _OPS and t.dtype != torch.bool))

    def allreduce_(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place all-reduce of the contiguous device tensor ``t`` on the current stream."""
        from ..ops import check

        assert t.is_contiguous() and self.supports(t, op)
        check(self.L.ha_comm_allreduce(self.handle, ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(t.data_ptr()),
                                       t.numel(), _DT[t.dtype], _OPS[op], self._stream(t)), "ha_comm_allreduce")
        return t

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        """[size, *t.shape] gathered blocks of equal shape."""
        from ..ops import check

        t = t.contiguous()
        out = torch.empty((self.size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        check(self.L.ha_comm_allgather(self.handle, ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                       t.numel(), _DT[t.dtype], self._stream(t)), "ha_comm_allgather")
        return out

    def reduce_scatter(self, inp: torch.Tensor, out: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """``out`` = this rank's block of the element-wise reduction of ``inp`` (size x out.numel()
        elements, contiguous) on the current stream."""
        from ..ops import check

        assert inp.is_contiguous() and out.is_contiguous() and self.supports(inp, op)
        assert inp.numel() == out.numel() * self.size and inp.dtype == out.dtype
        check(self.L.ha_comm_reducescatter(self.handle, ctypes.c_void_p(inp.data_ptr()),
                                           ctypes.c_void_p(out.data_ptr()), out.numel(), _DT[inp.dtype], _OPS[op],
                                           self._stream(inp)), "ha_comm_reducescatter")
        return out

    def allgatherv(self, moved: torch.Tensor, counts: Sequence[int]) -> torch.Tensor:
        """Concatenation along dim 0 of every rank's contiguous block (rank q holds counts[q]
        rows): one RCCL group of sends of the local block to every peer and receives of theirs,
        on the current stream (no padding to the largest block)."""
        from ..ops import check

        row = int(np.prod(moved.shape[1:])) * moved.element_size()
        out = torch.empty((sum(counts),) + tuple(moved.shape[1:]), dtype=moved.dtype, device=moved.device)
        sb, so, rb, ro = allgatherv_plan(counts, self.rank, row)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        check(self.L.ha_comm_alltoallv(self.handle, self.size, self.rank, ctypes.c_void_p(moved.data_ptr()), p(sb),
                                       p(so), ctypes.c_void_p(out.data_ptr()), p(rb), p(ro), self._stream(moved)),
              "ha_comm_alltoallv")
        return out

    def broadcast_(self, t: torch.Tensor, root: int) -> torch.Tensor:
        from ..ops import check

        assert t.is_contiguous()
        check(self.L.ha_comm_broadcast(self.handle, ctypes.c_void_p(t.data_ptr()), t.numel(), _DT[t.dtype], root,
                                       self._stream(t)), "ha_comm_broadcast")
        return t

    def alltoallv_bytes(self, send: torch.Tensor, send_bytes: Sequence[int], recv: torch.Tensor,
                        recv_bytes: Sequence[int]) -> torch.Tensor:
        """Personalised exchange of raw bytes (blocks back to back in rank order on both sides)."""
        from ..ops import check

        sb, so, rb, ro = alltoallv_plan(send_bytes, recv_bytes)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        ref = recv if recv.numel() else send
        check(self.L.ha_comm_alltoallv(self.handle, self.size, self.rank, ctypes.c_void_p(send.data_ptr()), p(sb),
                                       p(so), ctypes.c_void_p(recv.data_ptr()), p(rb), p(ro), self._stream(ref)),
              "ha_comm_alltoallv")
        return recv

    # ------------------------------------------------------------------ health
    def check(self) -> None:
        """Raise if RCCL reported an asynchronous error on this communicator (peer failure)."""
        e = self.L.ha_comm_async_error(self.handle)
        if e not in (0, 7):  # 7 = ncclInProgress (non-blocking init still running)
            raise RuntimeError("RCCL asynchronous error {} on the native communicator".format(e))

    def close(self, abort: bool = False) -> None:
        if getattr(self, "handle", None) is not None and self.handle.value:
            self.L.ha_comm_destroy(self.handle, int(abort))
            self.handle = None
