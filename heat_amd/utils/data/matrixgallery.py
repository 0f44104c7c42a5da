"""Test matrices (reference ``heat/utils/data/matrixgallery.py``: ``parter`` 15)."""
from __future__ import annotations

from ... import core as ht

__all__ = ["parter"]


def parter(n: int, split=None, device=None, comm=None, dtype=ht.float32):
    """The Parter matrix, a Toeplitz matrix with ``A[i, j] = 1 / (i - j + 0.5)`` (singular values
    cluster near pi)."""
    if split is None:
        a = ht.arange(n, dtype=dtype, device=device, comm=comm)
        I = ht.expand_dims(a, 0)
        J = ht.expand_dims(a, 1)
    elif split == 0:
        I = ht.expand_dims(ht.arange(n, dtype=dtype, device=device, comm=comm), 0)
        J = ht.expand_dims(ht.arange(n, dtype=dtype, split=0, device=device, comm=comm), 1)
    elif split == 1:
        I = ht.expand_dims(ht.arange(n, dtype=dtype, split=0, device=device, comm=comm), 0)
        J = ht.expand_dims(ht.arange(n, dtype=dtype, device=device, comm=comm), 1)
    else:
        raise ValueError("expected split value to be either {{None,0,1}}, but was {}".format(split))
    return 1.0 / (I - J + 0.5)
