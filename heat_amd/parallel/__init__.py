"""Process-group bootstrap, launcher and distributed primitives (ring pass, collectives helpers)."""
from . import backend
from .ring import ring_pass

__all__ = ["backend", "ring_pass"]
