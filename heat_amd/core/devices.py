"""
Device handling (reference ``heat/core/devices.py``: ``Device`` 17, ``cpu`` 79, ``gpu`` 98-115,
``get_device`` 121, ``sanitize_device`` 128, ``use_device`` 157).

MI355X-first: one process per GPU. The GPU bound to a process is ``LOCAL_RANK % device_count``
(the reference uses the global MPI rank, which is wrong on multi-node jobs); the launcher
(``heat_amd.run`` / ``torchrun``) sets ``LOCAL_RANK``.
"""
from __future__ import annotations

import os
from typing import Optional, Union

import torch

__all__ = ["Device", "cpu", "get_device", "sanitize_device", "use_device"]


class Device:
    """A compute device: ``device_type`` ('cpu'/'gpu'), ``device_id`` and the torch device string."""

    def __init__(self, device_type: str, device_id: int, torch_device: str):
        self.__device_type = device_type
        self.__device_id = device_id
        self.__torch_device = torch_device

    @property
    def device_type(self) -> str:
        return self.__device_type

    @property
    def device_id(self) -> int:
        return self.__device_id

    @property
    def torch_device(self) -> str:
        return self.__torch_device

    def __repr__(self) -> str:
        return "device({})".format(self.__str__())

    def __str__(self) -> str:
        return "{}:{}".format(self.device_type, self.device_id)

    def __eq__(self, other) -> bool:
        if isinstance(other, Device):
            return self.device_type == other.device_type and self.device_id == other.device_id
        if isinstance(other, torch.device):
            return self.device_type == ("gpu" if other.type == "cuda" else other.type)
        return NotImplemented

    def __hash__(self):
        return hash((self.device_type, self.device_id))


cpu = Device("cpu", 0, "cpu")
"""The standard CPU device."""

__default_device = cpu

if torch.cuda.device_count() > 0:
    _local = int(os.environ.get("LOCAL_RANK", os.environ.get("OMPI_COMM_WORLD_LOCAL_RANK", "0")))
    _gpu_id = _local % torch.cuda.device_count()
    gpu = Device("gpu", _gpu_id, "cuda:{}".format(_gpu_id))
    """The GPU bound to this process (one process per MI355X)."""
    __all__.append("gpu")
    if os.environ.get("HEAT_AMD_DEFAULT_DEVICE", "cpu").lower() in ("gpu", "cuda"):
        __default_device = gpu


def get_device() -> Device:
    """The currently configured default device."""
    return __default_device


def sanitize_device(device: Optional[Union[str, Device]] = None) -> Device:
    """Map a device specifier ('cpu', 'gpu', 'cuda', 'cuda:0', Device, None) to a Device."""
    if isinstance(device, Device):
        return device
    if device is None:
        return get_device()
    if isinstance(device, torch.device):
        device = device.type
    if isinstance(device, str):
        d = device.strip().lower()
        if d.startswith("cpu"):
            return cpu
        if d.startswith("gpu") or d.startswith("cuda"):
            if "gpu" not in globals():
                raise ValueError("Unknown device, must be one of {}".format(", ".join(_available())))
            return globals()["gpu"]
    raise ValueError("Unknown device, must be one of {}".format(", ".join(_available())))


def _available():
    return ["cpu"] + (["gpu"] if "gpu" in globals() else [])


def use_device(device: Optional[Union[str, Device]] = None) -> None:
    """Set the default device used by all factories."""
    global __default_device
    __default_device = sanitize_device(device)
    if __default_device.device_type == "gpu":
        torch.cuda.set_device(__default_device.device_id)


def _device_of_tensor(t: torch.Tensor) -> Device:
    if t.is_cuda and "gpu" in globals():
        return globals()["gpu"]
    return cpu
