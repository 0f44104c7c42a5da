"""
Native CDNA4 (gfx950) kernels and their Python entry points.

``heat_amd.ops`` is the only place where device compute leaves PyTorch: the hot paths of the
framework (k-means assign/update, pairwise distances, statistical moments, Threefry RNG, ...)
are hand-written HIP kernels in ``csrc/`` compiled into ``_lib/libheat_amd_kernels.so``.

Dispatch rule: a CUDA (= HIP) tensor ALWAYS goes to the native kernel; if the library cannot be
loaded on a GPU process this raises (set ``HEAT_AMD_ALLOW_FALLBACK=1`` to permit the PyTorch
reference path instead). Host tensors use the PyTorch reference implementation, which is also
the numerics oracle in the tests.
"""
from __future__ import annotations

import ctypes
import os
import warnings
import threading

import torch

from . import _build

_lib = None
_lock = threading.Lock()
_load_error = None

c_void_p, c_int, c_int64, c_double = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double

_SIGNATURES = {
    "ha_km_workspace_floats": (c_int, [c_int, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
    "ha_km_assign": (c_int, [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int, c_int64, c_void_p, c_void_p,
                             c_void_p, c_void_p]),
    "ha_km_update_workspace": (c_int64, [c_int64, c_int, c_int, c_int]),
    "ha_km_update": (c_int, [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                             c_int, c_void_p]),
    "ha_moments_rows": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p, c_int, c_double,
                                c_void_p, c_void_p]),
    "ha_moments_cols": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p, c_int, c_double,
                                c_void_p, c_void_p]),
}


def _optional_signatures():
    """Signatures of kernels added in later files (registered if the symbol exists)."""
    from . import signatures

    return signatures.SIGNATURES


def lib():
    """Load (building first if the sources are newer) the native kernel library."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        try:
            path = _build.LIBPATH
            if _build.needs_build():
                try:
                    path = _build.build()
                except Exception as e:
                    # a prebuilt library exists but is OLDER than the sources: using it may call a
                    # changed C signature with the old ABI. Say so loudly (naming what failed), and
                    # refuse under HEAT_STRICT_BUILD=1.
                    if not os.path.exists(_build.LIBPATH) or os.environ.get("HEAT_STRICT_BUILD") == "1":
                        raise
                    stale = [os.path.basename(s) for s in _build.stale_sources()]
                    warnings.warn("heat_amd: rebuilding the native kernels failed ({}); loading the STALE "
                                  "library {} (older than {}). Kernels whose C signature changed may be "
                                  "called with the wrong ABI.".format(str(e).strip()[:2000], _build.LIBPATH,
                                                                       ", ".join(stale) or "the build script"),
                                  RuntimeWarning, stacklevel=2)
            handle = ctypes.CDLL(path)
            sigs = dict(_SIGNATURES)
            try:
                sigs.update(_optional_signatures())
            except ImportError:
                pass
            for name, (res, args) in sigs.items():
                if hasattr(handle, name):
                    fn = getattr(handle, name)
                    fn.restype = res
                    fn.argtypes = args
            _lib = handle
        except Exception as e:
            _load_error = e
            raise
    return _lib


def available() -> bool:
    """Whether the native kernel library can be loaded (the load error is kept for the messages)."""
    try:
        lib()
        return True
    except Exception:
        return False


def allow_fallback() -> bool:
    """Whether ``HEAT_AMD_ALLOW_FALLBACK=1`` lets device tensors fall back to torch when the native
    library is missing (off by default: a missing library on a GPU box is an error)."""
    return os.environ.get("HEAT_AMD_ALLOW_FALLBACK", "0") == "1"


def use_native(t: torch.Tensor) -> bool:
    """True if ``t`` must be processed by the native kernels (device tensor). Raises if the
    library is unavailable on a device tensor and fallback is not explicitly allowed."""
    if not t.is_cuda:
        return False
    if available():
        return True
    if allow_fallback():
        return False
    raise RuntimeError("heat_amd native kernel library is not available for a device tensor: {}".format(_load_error))


# HEAT_DEBUG_STREAMS=1: remember the stream of the last native launch per device so that a
# collective issued on ANOTHER stream while that one still has work queued is reported as the
# race it is (see ``core.communication.MPICommunication._check_stream``)
DEBUG_STREAMS = os.environ.get("HEAT_DEBUG_STREAMS", "0") == "1"
LAST_LAUNCH_STREAM = {}


def stream_ptr(device=None) -> int:
    """The raw HIP stream handle of the current torch stream of ``device`` (for the ctypes launches)."""
    s = torch.cuda.current_stream(device)
    if DEBUG_STREAMS:
        LAST_LAUNCH_STREAM[s.device.index] = s
    return s.cuda_stream


def check(rc: int, name: str):
    """Raise RuntimeError naming ``name`` when a native entry point returned a non-zero status."""
    if rc != 0:
        raise RuntimeError("native kernel {} failed with status {}".format(name, rc))


from .kernels import *  # noqa: E402,F401,F403
