"""Process-group bootstrap, launcher and distributed primitives (ring pass, collectives helpers)."""
from . import backend
from .guard import RemoteRankError, collective_guard, exception_barrier
from .ring import ring_pass

__all__ = ["backend", "ring_pass", "collective_guard", "exception_barrier", "RemoteRankError"]
