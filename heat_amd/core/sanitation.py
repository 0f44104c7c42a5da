"""Input/output validation helpers (reference ``heat/core/sanitation.py``: ``sanitize_in`` 30,
``sanitize_infinity`` 50, ``sanitize_lshape`` 87, ``sanitize_out`` 139, ``sanitize_sequence`` 174,
``scalar_to_1d`` 196)."""
from __future__ import annotations

from typing import Any, List, Sequence, Tuple, Union

import torch

from .dndarray import DNDarray

__all__ = ["sanitize_in", "sanitize_infinity", "sanitize_in_tensor", "sanitize_lshape",
           "sanitize_out", "sanitize_sequence", "scalar_to_1d"]


def sanitize_in(x: Any):
    """Raise TypeError unless ``x`` is a DNDarray."""
    if not isinstance(x, DNDarray):
        raise TypeError("Input must be a DNDarray, is {}".format(type(x)))


def sanitize_infinity(x: Union[DNDarray, torch.Tensor]) -> Union[int, float]:
    """Largest representable value of the array's dtype (a finite stand-in for infinity)."""
    dtype = x.dtype if isinstance(x, torch.Tensor) else x.larray.dtype
    if dtype.is_floating_point:
        return torch.finfo(dtype).max
    if dtype == torch.bool:
        return True
    return torch.iinfo(dtype).max


def sanitize_in_tensor(x: Any):
    if not isinstance(x, torch.Tensor):
        raise TypeError("Input must be a torch.Tensor, is {}".format(type(x)))


def sanitize_lshape(array: DNDarray, tensor: torch.Tensor):
    """Check that a local tensor is a valid process-local chunk of ``array``."""
    tshape = tuple(tensor.shape)
    if tshape == array.lshape:
        return
    gshape, split = array.gshape, array.split
    if split is None:
        nz = [i for i, s in enumerate(tshape) if s != 0]
        if all(tshape[i] == gshape[i] for i in nz):
            return
        raise ValueError("Shape of local tensor is inconsistent with global DNDarray: tensor.shape is {}, should be {}"
                         .format(tshape, gshape))
    if tshape[:split] + tshape[split + 1:] == gshape[:split] + gshape[split + 1:]:
        return
    raise ValueError("Shape of local tensor along non-split axes is inconsistent with global DNDarray: "
                     "tensor.shape is {}, DNDarray is {}".format(tshape, gshape))


def sanitize_out(out: Any, output_shape: Tuple, output_split: int, output_device, output_comm=None):
    """Validate an ``out=`` buffer against the expected global shape, split and device."""
    if not isinstance(out, DNDarray):
        raise TypeError("expected `out` to be None or a DNDarray, but was {}".format(type(out)))
    if tuple(out.gshape) != tuple(output_shape):
        raise ValueError("Expecting output buffer of shape {}, got {}".format(output_shape, out.shape))
    if out.split != output_split:
        raise ValueError("Split axis of output buffer is inconsistent with split semantics (see documentation).")
    if output_device is not None:
        from .devices import sanitize_device

        output_device = sanitize_device(output_device)
    if output_device is not None and out.device != output_device:
        raise ValueError("Device mismatch: out is on {}, should be on {}".format(out.device, output_device))


def sanitize_sequence(seq) -> List:
    if isinstance(seq, list):
        return seq
    if isinstance(seq, tuple):
        return list(seq)
    raise TypeError("seq must be a list or a tuple, got {}".format(type(seq)))


def scalar_to_1d(x: DNDarray) -> DNDarray:
    """Turn a 0-d DNDarray into a 1-element 1-d DNDarray."""
    from . import factories

    return factories.array(x.larray.unsqueeze(0), dtype=x.dtype, split=x.split, comm=x.comm, device=x.device)
