"""
Parallel counter-based random number generation, bit-exact with the reference's Threefry
(``heat/core/random.py``: counter sequence 55-200, ``get_state`` 203, float conversion 220-245,
Kundu normal transform 248, ``normal`` 268, ``permutation`` 326, ``rand`` 396, ``randint`` 473,
``randn`` 580, ``randperm`` 637, ``seed`` 760, ``set_state`` 778, ``standard_normal`` 815,
``__threefry32/64`` 864/966 with only 8 of 12 rounds active).

On the GPU the whole chain (counter -> 8 Threefry rounds -> float / normal / integer) is ONE
native kernel (``ops/csrc/threefry.hip``); on the CPU a vectorised torch implementation of the
same arithmetic produces identical bits.

Layout semantics (kept exactly): the rank's local block consumes the contiguous range of the
flat random stream of length ``numel / shape[split] * counts[rank]`` that starts after the
lower ranks' ranges, and is reshaped to the local shape.
"""
from __future__ import annotations

import time
from typing import List, Optional, Tuple, Union

import numpy as np
import torch

from . import communication, devices, factories, types
from .communication import sanitize_comm
from .dndarray import DNDarray
from .stride_tricks import sanitize_axis, sanitize_shape
from .. import ops

__all__ = ["get_state", "normal", "permutation", "rand", "ranf", "randint", "random_integer", "randn", "random",
           "random_sample", "randperm", "sample", "seed", "set_state", "standard_normal"]

__seed: int = None
__counter: int = None

_M32 = 0xFFFFFFFF
_M64 = 0xFFFFFFFFFFFFFFFF
_M128 = (1 << 128) - 1
_DIST = {"uniform": 0, "normal": 1, "int": 2}


# ---------------------------------------------------------------------------------------------
# torch reference implementation (host tensors): uint32 / uint64 arithmetic emulated on int64
# ---------------------------------------------------------------------------------------------
def _rotl32(x, r):
    return ((x << r) | (x >> (32 - r))) & _M32


def _threefry32_t(x0: torch.Tensor, x1: torch.Tensor, key: int):
    k = key & 0x7FFFFFFF
    ks0 = ks1 = k
    ks2 = 466688986 ^ k ^ k
    x0 = (x0 + ks0) & _M32
    x1 = (x1 + ks1) & _M32
    for r in (13, 15, 26, 6):
        x0 = (x0 + x1) & _M32
        x1 = _rotl32(x1, r) ^ x0
    x0 = (x0 + ks1) & _M32
    x1 = (x1 + ks2 + 1) & _M32
    for r in (17, 29, 16, 24):
        x0 = (x0 + x1) & _M32
        x1 = _rotl32(x1, r) ^ x0
    x0 = (x0 + ks0) & _M32
    x1 = (x1 + ks1 + 3) & _M32
    return x0, x1


def _lshr64(x: torch.Tensor, r: int) -> torch.Tensor:
    return (x >> r) & ((1 << (64 - r)) - 1)


def _rotl64(x, r):
    return (x << r) | _lshr64(x, 64 - r)


def _to_signed64(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


def _threefry64_t(x0: torch.Tensor, x1: torch.Tensor, key: int):
    ks0 = ks1 = _to_signed64(key)
    ks2 = _to_signed64(2004413935125273122 ^ (key & _M64) ^ (key & _M64))
    x0 = x0 + ks0
    x1 = x1 + ks1
    for r in (16, 42, 12, 31):
        x0 = x0 + x1
        x1 = _rotl64(x1, r) ^ x0
    x0 = x0 + ks1
    x1 = x1 + _to_signed64(ks2 + 1)
    for r in (16, 32, 24, 21):
        x0 = x0 + x1
        x1 = _rotl64(x1, r) ^ x0
    x0 = x0 + ks0
    x1 = x1 + _to_signed64(ks1 + 3)
    return x0, x1


def _fill_torch(e0: int, n: int, counter: int, key: int, bits: int, dist: str, low: int, span: int, device):
    p0, p1 = e0 >> 1, (e0 + n + 1) >> 1
    g = torch.arange(p0, p1, dtype=torch.int64, device=device)
    if bits == 32:
        base = counter & _M64
        hi0, lo0 = base >> 32, base & _M32
        lo = g + lo0
        x1 = lo & _M32
        x0 = ((lo >> 32) + hi0) & _M32
        x0, x1 = _threefry32_t(x0, x1, key)
        vals = torch.stack([x0, x1], dim=1).reshape(-1)
        vals = vals[e0 - 2 * p0: e0 - 2 * p0 + n]
        if dist == "int":
            s = torch.where(vals >= (1 << 31), vals - (1 << 32), vals).to(torch.int32)
            a = torch.abs(s).to(torch.int64)
            return (torch.remainder(a, span) + low).to(torch.int32)
        u = (vals & 0x7FFFFF).to(torch.float32) * (1.0 / 8388608.0)
        return _kundu(u) if dist == "normal" else u
    base_lo, base_hi = counter & _M64, (counter >> 64) & _M64
    # lo = base_lo + g with carry into hi (uint64 emulated on int64 with wrap)
    lo_u = torch.tensor(_to_signed64(base_lo), dtype=torch.int64, device=device) + g
    # carry when the unsigned sum wraps: unsigned(lo) < unsigned(base_lo)
    flip = torch.tensor(-(1 << 63), dtype=torch.int64, device=device)
    carry = ((lo_u ^ flip) < (torch.tensor(_to_signed64(base_lo), dtype=torch.int64, device=device) ^ flip)).to(torch.int64)
    x0 = torch.full_like(g, _to_signed64(base_hi)) + carry
    x1 = lo_u
    x0, x1 = _threefry64_t(x0, x1, key)
    vals = torch.stack([x0, x1], dim=1).reshape(-1)[e0 - 2 * p0: e0 - 2 * p0 + n]
    if dist == "int":
        a = torch.abs(vals)
        return torch.remainder(a, span) + low
    u = (vals & 0x1FFFFFFFFFFFFF).to(torch.float64) * (1.0 / 9007199254740992.0)
    return _kundu(u) if dist == "normal" else u


_KUNDU_TABLE_DEVICES = set()


def _ensure_kundu_table(L, tdev) -> None:
    """Upload (once per device) the host-computed Kundu values for u within 2^-5 of 1, where the
    device's fast transform defers to them (``ops/csrc/threefry.hip``): computed with THIS module's
    torch formula, so the device matches the host path exactly where rounding decides the value."""
    import ctypes

    idx = tdev.index if tdev.index is not None else torch.cuda.current_device()
    if idx in _KUNDU_TABLE_DEVICES:
        return
    count = L.ha_threefry_kundu_table_size()
    v23 = 8388607 - torch.arange(count, dtype=torch.int64)
    tab = _kundu(v23.to(torch.float32) * (1.0 / 8388608.0)).to(torch.float32).contiguous()
    with torch.cuda.device(idx):
        rc = L.ha_threefry_set_kundu_table(ctypes.c_void_p(tab.data_ptr()), count)
    if rc != 0:
        raise RuntimeError("uploading the Kundu table failed (code {})".format(rc))
    _KUNDU_TABLE_DEVICES.add(idx)


def _kundu(values: torch.Tensor) -> torch.Tensor:
    inner = 1 - values ** 0.0775
    tiny = torch.finfo(inner.dtype).tiny
    return (torch.log(-torch.log(inner + tiny) + tiny) - 1.0821) * (1.0 / 0.3807)


# ---------------------------------------------------------------------------------------------
# counter bookkeeping
# ---------------------------------------------------------------------------------------------
def _local_range(shape, split, comm) -> Tuple[int, int, tuple]:
    """(first global stream element, number of local elements, local shape)."""
    total = int(np.prod(shape)) if len(shape) else 1
    if split is None:
        return 0, total, tuple(shape)
    counts, _, _ = comm.counts_displs_shape(shape, split)
    per = total // shape[split] if shape[split] else 0
    e0 = per * sum(counts[: comm.rank])
    _, lshape, _ = comm.chunk(shape, split)
    return e0, per * counts[comm.rank], lshape


def _generate(shape, dtype, split, device, comm, dist: str, low: int = 0, span: int = 1) -> DNDarray:
    global __counter
    shape = tuple(int(s) for s in shape)
    split = sanitize_axis(shape, split)
    device = devices.sanitize_device(device)
    comm = sanitize_comm(comm)
    ttype = dtype.torch_type()
    bits = 32 if ttype in (torch.float32, torch.int32) else 64
    total = int(np.prod(shape)) if len(shape) else 1
    if bits == 32 and total > 2 * _M32:
        raise ValueError("Shape is to big with {} elements".format(total))
    e0, n, lshape = _local_range(shape, split, comm)
    counter = __counter
    tdev = torch.device(device.torch_device)
    out = torch.empty(n, dtype=ttype, device=tdev)
    if n > 0:
        if ops.use_native(out):
            from ..ops import lib, stream_ptr, check
            import ctypes

            L = lib()
            if bits == 32 and dist == "normal":
                _ensure_kundu_table(L, tdev)
            rc = L.ha_threefry_fill(ctypes.c_void_p(out.data_ptr()), e0, n, counter & _M64, (counter >> 64) & _M64,
                                    __seed & _M64, bits, _DIST[dist], float(low), float(span),
                                    ctypes.c_void_p(stream_ptr(tdev)))
            check(rc, "ha_threefry_fill")
        else:
            out = _fill_torch(e0, n, counter, __seed, bits, dist, low, span, tdev).to(ttype)
    __counter = (counter + (total + 1) // 2) & _M128
    return DNDarray(out.reshape(lshape), shape, dtype, split, device, comm, True)


# ---------------------------------------------------------------------------------------------
# public API
# ---------------------------------------------------------------------------------------------
def get_state() -> Tuple[str, int, int, int, float]:
    """('Threefry', seed, counter, 0, 0.0)."""
    return "Threefry", __seed, __counter, 0, 0.0


def set_state(state: Tuple[str, int, int, int, float]):
    """Set (seed, counter) from a state tuple returned by :func:`get_state`."""
    if not isinstance(state, tuple) or (len(state) != 3 and len(state) != 5):
        raise TypeError("state needs to be a three- or five-tuple")
    if state[0] != "Threefry":
        raise ValueError("algorithm must be 'Threefry'")
    global __seed, __counter
    __seed = int(state[1])
    __counter = int(state[2])


def seed(seed: Optional[int] = None):
    """Seed the generator (time-based, broadcast from rank 0, if None); also seeds torch."""
    if seed is None:
        seed = communication.MPI_WORLD.bcast(int(time.time() * 256))
    global __seed, __counter
    __seed = seed
    __counter = 0
    torch.manual_seed(seed)


def _shape_from_args(args):
    if not args:
        return (1,)
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = tuple(args[0])
    try:
        shape = tuple(int(a) for a in args)
    except (TypeError, ValueError):
        raise TypeError("dimensions must be integers")
    if not all(s > 0 for s in shape):
        raise ValueError("negative dimensions are not allowed")
    return shape


def rand(*args, dtype=types.float32, split: Optional[int] = None, device=None, comm=None) -> DNDarray:
    """Uniform samples over [0, 1) of the given shape."""
    shape = _shape_from_args(args)
    dtype = types.canonical_heat_type(dtype)
    if dtype not in (types.float32, types.float64):
        raise ValueError("dtype is none of ht.float32 or ht.float64 but was {}".format(dtype))
    return _generate(shape, dtype, split, device, comm, "uniform")


def randn(*args, dtype=types.float32, split: Optional[int] = None, device=None, comm=None) -> DNDarray:
    """Standard-normal samples (Kundu transform of :func:`rand`)."""
    shape = _shape_from_args(args)
    dtype = types.canonical_heat_type(dtype)
    if dtype not in (types.float32, types.float64):
        raise ValueError("dtype is none of ht.float32 or ht.float64 but was {}".format(dtype))
    return _generate(shape, dtype, split, device, comm, "normal")


def randint(low: int, high: Optional[int] = None, size=None, dtype=types.int32, split: Optional[int] = None,
            device=None, comm=None) -> DNDarray:
    """Integers in [low, high) (documented modulo bias, like the reference)."""
    if high is None:
        low, high = 0, low
    if not isinstance(low, (int, np.integer)) or not isinstance(high, (int, np.integer)):
        raise TypeError("low and high must be integers")
    span = int(high) - int(low)
    if span <= 0:
        raise ValueError("low >= high")
    if size is None:
        size = (1,)
    shape = tuple(sanitize_shape(size))
    if not all(s > 0 for s in shape):
        raise ValueError("negative dimensions are not allowed")
    dtype = types.canonical_heat_type(dtype)
    if dtype not in (types.int32, types.int64):
        raise ValueError("Unsupported dtype for randint")
    return _generate(shape, dtype, split, device, comm, "int", int(low), span)


def random_integer(low, high=None, size=None, dtype=types.int32, split=None, device=None, comm=None) -> DNDarray:
    return randint(low, high, size, dtype, split, device, comm)


def random(shape=None, dtype=types.float32, split=None, device=None, comm=None) -> DNDarray:
    """Uniform samples over [0, 1) of ``shape``."""
    if shape is None:
        shape = (1,)
    shape = sanitize_shape(shape)
    return rand(*shape, dtype=dtype, split=split, device=device, comm=comm)


random_sample = ranf = sample = random


def standard_normal(shape=None, dtype=types.float32, split=None, device=None, comm=None) -> DNDarray:
    if shape is None:
        shape = (1,)
    shape = sanitize_shape(shape)
    return randn(*shape, dtype=dtype, split=split, device=device, comm=comm)


def normal(mean=0.0, std=1.0, shape=None, dtype=types.float32, split=None, device=None, comm=None) -> DNDarray:
    """Normal samples with ``mean`` and ``std`` (scalars or DNDarrays)."""
    if not (isinstance(mean, (int, float)) or isinstance(mean, DNDarray)):
        raise TypeError("'mean' must be float or DNDarray")
    if not (isinstance(std, (int, float)) or isinstance(std, DNDarray)):
        raise TypeError("'std' must be float or DNDarray")
    if isinstance(std, (int, float)) and std < 0:
        raise ValueError("'std' must be non-negative")
    if isinstance(std, DNDarray):
        from . import logical

        if logical.any(std < 0):
            raise ValueError("'std' must be non-negative")
    if shape is None:
        shape = mean.shape if isinstance(mean, DNDarray) else (std.shape if isinstance(std, DNDarray) else (1,))
    shape = sanitize_shape(shape)
    return mean + std * randn(*shape, dtype=dtype, split=split, device=device, comm=comm)


def randperm(n: int, dtype=types.int64, split: Optional[int] = None, device=None, comm=None) -> DNDarray:
    """Random permutation of ``range(n)`` (torch generator, identical on every rank)."""
    if not isinstance(n, (int, np.integer)):
        raise TypeError("n must be int, currently {}".format(type(n)))
    dtype = types.canonical_heat_type(dtype)
    device = devices.sanitize_device(device)
    perm = torch.randperm(int(n), dtype=dtype.torch_type(), device=device.torch_device)
    return factories.array(perm, dtype=dtype, device=device, split=split, comm=comm)


def permutation(x) -> DNDarray:
    """Randomly permute a sequence / array along axis 0 (one personalised exchange)."""
    if isinstance(x, (int, np.integer)):
        return randperm(int(x))
    if not isinstance(x, DNDarray):
        raise TypeError("x must be int or DNDarray")
    perm = torch.randperm(x.gshape[0], device=x.larray.device)
    return x[perm]


# roll a time-based seed at import (collective when distributed, like the reference)
seed()
