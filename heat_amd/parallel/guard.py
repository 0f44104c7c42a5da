"""
Failure propagation for SPMD code (the reference only does this inside
``save_netcdf``, ``heat/core/io.py:593-650``).

``collective_guard(comm)`` wraps a block that may fail on SOME ranks (I/O, user callbacks,
data-dependent checks): at the end of the block all ranks exchange a failure flag and every rank
raises (the failing rank its own exception, the others a ``RemoteRankError`` naming it), instead
of the healthy ranks deadlocking in the next collective. Hangs that are not exceptions are
bounded by the process-group timeout (``HEAT_COMM_TIMEOUT``) with RCCL's asynchronous error
handling enabled at initialisation (``parallel.backend``).
"""
from __future__ import annotations

import contextlib
from typing import Optional

__all__ = ["RemoteRankError", "collective_guard", "exception_barrier"]


class RemoteRankError(RuntimeError):
    """Raised on healthy ranks when another rank failed inside a guarded block."""

    def __init__(self, rank: int, what: str):
        super().__init__("rank {} failed: {}".format(rank, what))
        self.rank = rank
        self.what = what


def exception_barrier(comm, exc: Optional[BaseException]) -> None:
    """Collective: re-raise ``exc`` locally, or a :class:`RemoteRankError` if another rank failed."""
    flags = comm.allgather(None if exc is None else "{}: {}".format(type(exc).__name__, exc))
    bad = [(r, f) for r, f in enumerate(flags) if f is not None]
    if bad:
        if exc is not None:
            raise exc
        raise RemoteRankError(bad[0][0], bad[0][1])


@contextlib.contextmanager
def collective_guard(comm=None):
    """``with collective_guard(comm): ...`` - see the module docstring."""
    from ..core.communication import sanitize_comm

    comm = sanitize_comm(comm)
    try:
        yield
    except BaseException as e:  # noqa: B902 - re-raised after the exchange
        exception_barrier(comm, e)
        raise
    exception_barrier(comm, None)
