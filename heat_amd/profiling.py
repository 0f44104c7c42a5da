"""
Tracing, counters, fault injection and logging (the reference has none of this).

* ``enable()`` (or ``HEAT_TRACE=1`` at import) wraps every collective of
  :class:`~heat_amd.core.communication.MPICommunication` and every native kernel entry point of
  :mod:`heat_amd.ops` with a roctx range (visible in ``rocprofv3 --marker-trace`` / rocprof
  timelines) and accumulates per-op counters: calls, bytes moved, device time (HIP events when
  ``timing=True``).
* ``counters()`` returns them as a dict (JSON-serialisable) - benchmarks attach it to results.
* ``HEAT_DEBUG_COLLECTIVES=1``: every collective first all-gathers an (op, dtype) signature and
  aborts on mismatch (catches divergent SPMD control flow, see ``communication._trace``).
* ``HEAT_FAULT_INJECT="rank:op:n"``: raise on the n-th call of collective ``op`` on ``rank`` (for
  testing failure propagation).
* ``log``: rank-prefixed logger (rank 0 only unless ``HEAT_LOG_ALL_RANKS=1``).
"""
from __future__ import annotations

import contextlib
import functools
import json
import logging
import os
import sys
import time
from collections import defaultdict
from typing import Dict

import torch

__all__ = ["enable", "disable", "enabled", "counters", "reset", "region", "log", "dump"]

_COLLECTIVES = ["Allreduce", "Iallreduce", "Bcast", "Ibcast", "Allgather", "Allgatherv", "Iallgather", "Iallgatherv",
                "Alltoall", "Alltoallv", "Gatherv", "Scatterv", "Exscan", "Scan", "Reduce", "Send", "Recv", "Isend",
                "Irecv", "exchange", "allgather_tensor", "Barrier", "bcast", "allgather", "allreduce"]
_KERNELS = ["kmeans_assign", "kmeans_update", "kmeans_step_small", "moments", "cdist", "lasso_epoch", "knn_topk",
            "gemm_f16x3"]

_state = {"enabled": False, "timing": False, "originals": {}}
_counters: Dict[str, Dict[str, float]] = defaultdict(lambda: {"calls": 0, "bytes": 0, "ms": 0.0})
_fault = None
_fault_calls = defaultdict(int)


def _nbytes(args) -> int:
    total = 0
    for a in args:
        t = getattr(a, "larray", a)
        if isinstance(t, torch.Tensor):
            total += t.numel() * t.element_size()
        elif isinstance(a, (list, tuple)):
            total += _nbytes(a)
    return total


def _range_push(name: str):
    try:
        torch.cuda.nvtx.range_push(name)
        return True
    except Exception:
        return False


def _range_pop(pushed: bool):
    if pushed:
        try:
            torch.cuda.nvtx.range_pop()
        except Exception:
            pass


def _wrap(fn, name: str):
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        if _fault is not None:
            r, op, n = _fault
            rank = getattr(args[0], "rank", 0) if args else 0
            if op == name and rank == r:
                _fault_calls[name] += 1
                if _fault_calls[name] == n:
                    raise RuntimeError("HEAT_FAULT_INJECT: injected failure in {} (call {}) on rank {}"
                                       .format(name, n, rank))
        c = _counters[name]
        c["calls"] += 1
        c["bytes"] += _nbytes(args[1:] if args else ())
        pushed = _range_push("heat_amd." + name)
        timing = _state["timing"] and torch.cuda.is_available()
        if timing:
            start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            start.record()
        t0 = time.perf_counter()
        try:
            return fn(*args, **kwargs)
        finally:
            if timing:
                end.record()
                end.synchronize()
                c["ms"] += start.elapsed_time(end)
            else:
                c["ms"] += (time.perf_counter() - t0) * 1e3
            _range_pop(pushed)

    wrapper.__heat_wrapped__ = fn
    return wrapper


def enable(timing: bool = False) -> None:
    """Start tracing collectives and native kernels (``timing``: synchronous device timing)."""
    from .core.communication import MPICommunication
    from . import ops

    _state["timing"] = timing
    if _state["enabled"]:
        return
    for name in _COLLECTIVES:
        fn = getattr(MPICommunication, name, None)
        if fn is not None and not hasattr(fn, "__heat_wrapped__"):
            _state["originals"][("comm", name)] = fn
            setattr(MPICommunication, name, _wrap(fn, name))
    for name in _KERNELS:
        fn = getattr(ops, name, None)
        if fn is not None and not hasattr(fn, "__heat_wrapped__"):
            _state["originals"][("ops", name)] = fn
            setattr(ops, name, _wrap(fn, name))
    _state["enabled"] = True


def disable() -> None:
    """Undo ``enable``: restore the unwrapped communicator methods and native ops."""
    from .core.communication import MPICommunication
    from . import ops

    for (kind, name), fn in _state["originals"].items():
        setattr(MPICommunication if kind == "comm" else ops, name, fn)
    _state["originals"].clear()
    _state["enabled"] = False


def enabled() -> bool:
    """Whether the collective / native-op counters are being collected."""
    return _state["enabled"]


def counters() -> Dict[str, Dict[str, float]]:
    """A copy of the per-name counters collected since the last ``reset``."""
    return {k: dict(v) for k, v in _counters.items()}


def reset() -> None:
    """Clear all counters."""
    _counters.clear()


def dump(path: str) -> None:
    """Write ``counters()`` to ``path`` as JSON."""
    with open(path, "w") as f:
        json.dump(counters(), f, indent=1)


@contextlib.contextmanager
def region(name: str):
    """roctx range + wall-time counter around a block of user code."""
    pushed = _range_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        _counters["region:" + name]["calls"] += 1
        _counters["region:" + name]["ms"] += (time.perf_counter() - t0) * 1e3
        _range_pop(pushed)


def _make_logger() -> logging.Logger:
    lg = logging.getLogger("heat_amd")
    if not lg.handlers:
        rank = int(os.environ.get("RANK", "0"))
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("[heat_amd r{}] %(levelname)s %(message)s".format(rank)))
        lg.addHandler(h)
        if rank != 0 and os.environ.get("HEAT_LOG_ALL_RANKS", "0") != "1":
            lg.setLevel(logging.ERROR)
        else:
            lg.setLevel(os.environ.get("HEAT_LOG_LEVEL", "WARNING").upper())
    return lg


log = _make_logger()

_fi = os.environ.get("HEAT_FAULT_INJECT")
if _fi:
    try:
        _r, _op, _n = _fi.split(":")
        _fault = (int(_r), _op, int(_n))
    except ValueError:
        log.error("ignoring malformed HEAT_FAULT_INJECT=%s (expected rank:op:n)", _fi)


def _auto_enable() -> None:
    """Called at the end of ``heat_amd/__init__`` (after ops/communication exist)."""
    if os.environ.get("HEAT_TRACE", "0") == "1" or _fault is not None:
        enable(timing=os.environ.get("HEAT_TRACE_TIMING", "0") == "1")
