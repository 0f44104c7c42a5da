"""
Process-group bootstrap: one process per MI355X, ``torch.distributed`` with RCCL for device
buffers and gloo for host buffers (a single mixed-backend group ``cpu:gloo,cuda:nccl``).

Replaces the reference's implicit ``MPI_Init`` at import (``heat/core/communication.py:11``).
Rendezvous uses the standard ``MASTER_ADDR``/``MASTER_PORT``/``RANK``/``WORLD_SIZE`` environment
written by ``torchrun`` or by our own launcher (``python -m heat_amd.run -n N``). Without that
environment the process is a world of one and no process group is created at all.
"""
from __future__ import annotations

import atexit
import datetime
import os

import torch
import torch.distributed as dist

_INITIALISED_BY_US = False


def env_world() -> tuple:
    """(rank, world_size, local_rank) from the launcher environment (defaults: a world of one)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def backend_name() -> str:
    """Backend string for the world group. ``HEAT_COMM_BACKEND`` overrides (rccl|gloo|mixed)."""
    forced = os.environ.get("HEAT_COMM_BACKEND", "").lower()
    has_gpu = torch.cuda.device_count() > 0
    if forced == "gloo" or not has_gpu:
        return "gloo"
    if forced in ("rccl", "nccl"):
        return "nccl"
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", "0") or 0)
    if local_world > torch.cuda.device_count() and not forced:
        # more ranks on this node than GPUs: ranks would share a device, which RCCL refuses
        # ("Duplicate GPU detected") - run the world on gloo (device buffers host-staged)
        import warnings

        warnings.warn("{} local ranks on {} GPUs: ranks share devices, using the gloo backend".format(
            local_world, torch.cuda.device_count()))
        return "gloo"
    # device tensors -> RCCL over xGMI, host tensors (object collectives, CPU arrays) -> gloo
    return "cpu:gloo,cuda:nccl"


def ensure_initialized() -> bool:
    """Initialise the default process group if the environment describes a world > 1.

    Returns True when a (possibly pre-existing) process group is available.
    """
    global _INITIALISED_BY_US
    if dist.is_available() and dist.is_initialized():
        return True
    rank, world, local = env_world()
    if world <= 1 or not dist.is_available():
        return False
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    backend = backend_name()
    kwargs = {}
    if backend != "gloo":
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local % ndev)
    timeout = datetime.timedelta(seconds=int(os.environ.get("HEAT_COMM_TIMEOUT", "1800")))
    # watchdog: a collective that does not complete within the timeout aborts the communicator
    # and raises on every rank instead of hanging the job
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=timeout, **kwargs)
    _INITIALISED_BY_US = True
    atexit.register(shutdown)
    return True


def shutdown() -> None:
    """Destroy the process group if we created it (called at interpreter exit)."""
    global _INITIALISED_BY_US
    if _INITIALISED_BY_US and dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:
            pass
    _INITIALISED_BY_US = False
