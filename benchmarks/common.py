"""
Shared harness of the heat_amd benchmark suite (reference protocol: ``benchmarks/*/heat-gpu.py``,
re-done with correct device timing).

Every measurement is bracketed by ``torch.cuda.synchronize()`` + a barrier on both sides (the
reference reads ``time.perf_counter()`` without synchronising the device,
``benchmarks/kmeans/heat-gpu.py:25-27``), reports the MAX over ranks, and is printed by rank 0 as
one JSON line. Run one process per GPU: ``python -m heat_amd.run -n 8 benchmarks/kmeans/run.py``
or ``torchrun --nproc-per-node 8 --master-addr 127.0.0.1 ...``.
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Callable, Dict, List

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import heat_amd as ht  # noqa: E402


def setup() -> "ht.Device":
    if torch.cuda.is_available():
        ht.use_device("gpu")
    return ht.get_device()


def sync() -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    ht.MPI_WORLD.Barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def timed(fn: Callable[[], object], trials: int, warmup: int = 1) -> List[float]:
    """Wall seconds of ``trials`` calls (after ``warmup`` untimed ones), max over ranks."""
    for _ in range(warmup):
        fn()
    out = []
    for _ in range(trials):
        sync()
        t0 = time.perf_counter()
        fn()
        sync()
        dt = time.perf_counter() - t0
        out.append(ht.MPI_WORLD.allreduce(dt, ht.MPI.MAX) if ht.MPI_WORLD.size > 1 else dt)
    return out


def torch_reference(fn: Callable[[], object], trials: int, warmup: int = 1) -> List[float]:
    """Wall seconds of the reference's single-GPU torch comparator (``benchmarks/*/torch-gpu.py``
    of the reference: the same algorithm in plain torch on this process's data), timed with device
    synchronisation on both sides. Only meaningful in a world of one (the comparator is a 1-GPU
    protocol); returns [] otherwise."""
    if ht.MPI_WORLD.size != 1:
        return []
    for _ in range(warmup):
        fn()
    out = []
    for _ in range(trials):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        out.append(time.perf_counter() - t0)
    return out


def report(benchmark: str, case: Dict, times: List[float], work: Dict = None,
           reference: List[float] = None) -> Dict:
    """Rank 0 prints {benchmark, case, n_gpus, trials, median/min seconds, derived rates}; with
    ``reference`` (times of :func:`torch_reference`) also ``reference_torch_s`` (median) and
    ``speedup`` = reference median / this median."""
    times_sorted = sorted(times)
    med = times_sorted[len(times_sorted) // 2]
    rec = {"benchmark": benchmark, "case": case, "n_gpus": ht.MPI_WORLD.size,
           "device": "gpu" if torch.cuda.is_available() else "cpu", "trials": len(times),
           "median_s": med, "min_s": times_sorted[0], "times_s": times}
    for key, amount in (work or {}).items():
        rec[key] = amount / med
    if reference:
        ref = sorted(reference)[len(reference) // 2]
        rec["reference_torch_s"] = ref
        rec["speedup"] = ref / med if med > 0 else None
    if ht.MPI_WORLD.rank == 0:
        print(json.dumps(rec), flush=True)
    return rec
