"""
Parallel IO (reference ``heat/core/io.py``: ``load_hdf5`` 55, ``save_hdf5`` 147, ``load_netcdf`` 265,
``save_netcdf`` 348, ``load`` 659, ``load_csv`` 710, ``save`` 923).

* HDF5 / NetCDF: available when ``h5py`` / ``netCDF4`` are importable (same file layout as the
  reference; every rank reads only its hyperslab; writes are serialised rank by rank).
* CSV: every rank parses only its byte range; a line that straddles a boundary belongs to the
  rank where it starts, so no boundary repair messages are needed (the reference exchanges them,
  ``io.py:806-898``). Parsing uses pandas' C parser.
* ``.npy`` (our addition, no optional dependency): memory-mapped reads of the local hyperslab and
  in-place parallel writes into a pre-created file.
"""
from __future__ import annotations

import io as _io
import os
from typing import Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from . import devices, factories, types
from .communication import MPI, sanitize_comm
from .dndarray import DNDarray
from .stride_tricks import sanitize_axis

__all__ = ["load", "load_csv", "save", "save_csv", "load_npy", "save_npy", "supports_hdf5", "supports_netcdf"]

try:
    import h5py  # noqa: F401
except ImportError:
    h5py = None
try:
    import netCDF4 as nc  # noqa: F401
except ImportError:
    nc = None


def supports_hdf5() -> bool:
    return h5py is not None


def supports_netcdf() -> bool:
    return nc is not None


def _exception_barrier(comm, exc: Optional[BaseException]):
    """Propagate a failure on any rank to every rank (reference io.py:593-650, made generic)."""
    flags = comm.allgather(None if exc is None else repr(exc))
    bad = [(r, f) for r, f in enumerate(flags) if f is not None]
    if bad:
        if exc is not None:
            raise exc
        raise RuntimeError("rank {} failed: {}".format(bad[0][0], bad[0][1]))


# --------------------------------------------------------------------------------------------- npy
def load_npy(path: str, dtype=None, split: Optional[int] = None, device=None, comm=None) -> DNDarray:
    """Load a ``.npy`` file; each rank maps the file and copies only its hyperslab."""
    comm = sanitize_comm(comm)
    device = devices.sanitize_device(device)
    arr = np.load(path, mmap_mode="r", allow_pickle=False)
    gshape = tuple(arr.shape)
    split = sanitize_axis(gshape, split)
    _, _, sl = comm.chunk(gshape, split)
    local = np.array(arr[sl], copy=True)          # writable private copy of the mmap slice
    t = torch.from_numpy(local)
    htype = types.canonical_heat_type(dtype) if dtype is not None else types.canonical_heat_type(t.dtype)
    t = t.to(device=device.torch_device, dtype=htype.torch_type())
    return DNDarray(t, gshape, htype, split, device, comm, True)


def save_npy(data: DNDarray, path: str) -> None:
    """Write a DNDarray to ``.npy``: rank 0 creates the file, every rank writes its hyperslab."""
    comm = data.comm
    np_dtype = data.larray.cpu().numpy().dtype if data.larray.numel() else np.dtype(
        torch.empty(0, dtype=data.larray.dtype).numpy().dtype)
    exc = None
    if comm.rank == 0:
        try:
            mm = np.lib.format.open_memmap(path, mode="w+", dtype=np_dtype, shape=data.gshape)
            del mm
        except Exception as e:  # pragma: no cover - propagated below
            exc = e
    _exception_barrier(comm, exc)
    if data.split is None or not data.is_distributed():
        if comm.rank == 0:
            mm = np.lib.format.open_memmap(path, mode="r+")
            mm[...] = data.larray.cpu().numpy()
            mm.flush()
            del mm
    else:
        counts, displs = data.counts_displs()
        me = comm.rank
        if counts[me]:
            mm = np.lib.format.open_memmap(path, mode="r+")
            sl = [slice(None)] * data.ndim
            sl[data.split] = slice(displs[me], displs[me] + counts[me])
            mm[tuple(sl)] = data.larray.cpu().numpy()
            mm.flush()
            del mm
    comm.Barrier()


# --------------------------------------------------------------------------------------------- csv
def load_csv(path: str, header_lines: int = 0, sep: str = ",", dtype=types.float32, encoding: str = "utf-8",
             split: Optional[int] = None, device=None, comm=None) -> DNDarray:
    """Load a CSV file of numbers. With ``split=0`` every rank parses its byte range only."""
    if not isinstance(path, str):
        raise TypeError("path must be str, not {}".format(type(path)))
    if not isinstance(sep, str):
        raise TypeError("separator must be str, not {}".format(type(sep)))
    if not isinstance(header_lines, int):
        raise TypeError("header_line must int, not {}".format(type(header_lines)))
    if split not in (None, 0, 1):
        raise ValueError("split must be in [None, 0, 1], but is {}".format(split))
    comm = sanitize_comm(comm)
    device = devices.sanitize_device(device)
    htype = types.canonical_heat_type(dtype)
    import pandas as pd

    with open(path, "rb") as f:
        raw_header = b""
        for _ in range(header_lines):
            raw_header += f.readline()
        body_start = f.tell()
        f.seek(0, os.SEEK_END)
        size = f.tell()
    if split == 0 and comm.size > 1:
        body = size - body_start
        lo = body_start + body * comm.rank // comm.size
        hi = body_start + body * (comm.rank + 1) // comm.size
        with open(path, "rb") as f:
            # a line belongs to the rank in whose range it STARTS
            f.seek(lo)
            if lo > body_start:
                f.seek(lo - 1)
                prev = f.read(1)
                if prev != b"\n":
                    f.readline()
            start = f.tell()
            chunk = []
            pos = start
            while pos < hi:
                line = f.readline()
                if not line:
                    break
                chunk.append(line)
                pos += len(line)
            data = b"".join(chunk)
        if data.strip():
            df = pd.read_csv(_io.BytesIO(data), sep=sep, header=None, encoding=encoding, dtype=np.float64)
            local = torch.from_numpy(df.to_numpy())
        else:
            local = torch.empty((0, 0), dtype=torch.float64)
        ncols = comm.allreduce(int(local.shape[1]) if local.numel() else 0, MPI.MAX)
        if local.numel() == 0:
            local = torch.empty((0, ncols), dtype=torch.float64)
        local = local.to(device=device.torch_device, dtype=htype.torch_type())
        out = factories.array(local, is_split=0, device=device, comm=comm, dtype=htype)
        out.balance_()
        return out
    df = pd.read_csv(path, sep=sep, header=None, skiprows=header_lines, encoding=encoding, dtype=np.float64)
    t = torch.from_numpy(df.to_numpy()).to(device=device.torch_device, dtype=htype.torch_type())
    return factories.array(t, split=split, device=device, comm=comm, dtype=htype)


def save_csv(data: DNDarray, path: str, header_lines: Optional[List[str]] = None, sep: str = ",",
             decimals: int = -1, encoding: str = "utf-8", comm=None, truncate: bool = True) -> None:
    """Write a 1-D/2-D DNDarray as CSV (rank by rank, in order)."""
    comm = data.comm if comm is None else comm
    t = data
    if data.split == 1 and data.is_distributed():
        from .manipulations import resplit

        t = resplit(data, 0)
    rows = t.larray.cpu().numpy()
    if rows.ndim == 1:
        rows = rows.reshape(-1, 1)
    fmt = "%.{}f".format(decimals) if decimals >= 0 else "%s"
    for r in range(comm.size):
        if r == comm.rank and (t.is_distributed() or comm.rank == 0):
            mode = "w" if (r == 0 and truncate) else "a"
            with open(path, mode, encoding=encoding) as f:
                if r == 0 and header_lines:
                    for h in header_lines:
                        f.write(h.rstrip("\n") + "\n")
                if rows.size:
                    np.savetxt(f, rows, delimiter=sep, fmt=fmt)
        comm.Barrier()


# --------------------------------------------------------------------------------------------- hdf5
if h5py is not None:
    __all__ += ["load_hdf5", "save_hdf5"]

    def load_hdf5(path: str, dataset: str, dtype=types.float32, load_fraction: float = 1.0,
                  split: Optional[int] = None, device=None, comm=None) -> DNDarray:
        """Load an HDF5 dataset; every rank reads only its hyperslab."""
        comm = sanitize_comm(comm)
        device = devices.sanitize_device(device)
        htype = types.canonical_heat_type(dtype)
        with h5py.File(path, "r") as handle:
            data = handle[dataset]
            gshape = list(data.shape)
            if split is not None:
                gshape[split] = int(gshape[split] * load_fraction)
            gshape = tuple(gshape)
            split = sanitize_axis(gshape, split)
            _, _, sl = comm.chunk(gshape, split)
            local = torch.tensor(np.asarray(data[sl]), dtype=htype.torch_type(), device=device.torch_device)
        return DNDarray(local, gshape, htype, split, device, comm, True)

    def save_hdf5(data: DNDarray, path: str, dataset: str, mode: str = "w", **kwargs) -> None:
        """Write a DNDarray into an HDF5 dataset (rank by rank)."""
        comm = data.comm
        if comm.rank == 0:
            with h5py.File(path, mode) as handle:
                handle.create_dataset(dataset, data.gshape, dtype=data.larray.cpu().numpy().dtype, **kwargs)
        comm.Barrier()
        if data.split is None or not data.is_distributed():
            if comm.rank == 0:
                with h5py.File(path, "r+") as handle:
                    handle[dataset][...] = data.larray.cpu().numpy()
            comm.Barrier()
            return
        counts, displs = data.counts_displs()
        for r in range(comm.size):
            if r == comm.rank and counts[r]:
                with h5py.File(path, "r+") as handle:
                    sl = [slice(None)] * data.ndim
                    sl[data.split] = slice(displs[r], displs[r] + counts[r])
                    handle[dataset][tuple(sl)] = data.larray.cpu().numpy()
            comm.Barrier()

    DNDarray.save_hdf5 = lambda self, path, dataset, mode="w", **kwargs: save_hdf5(self, path, dataset, mode, **kwargs)

# --------------------------------------------------------------------------------------------- netcdf
if nc is not None:
    __all__ += ["load_netcdf", "save_netcdf"]

    def load_netcdf(path: str, variable: str, dtype=types.float32, split: Optional[int] = None, device=None,
                    comm=None) -> DNDarray:
        comm = sanitize_comm(comm)
        device = devices.sanitize_device(device)
        htype = types.canonical_heat_type(dtype)
        with nc.Dataset(path, "r") as handle:
            data = handle[variable]
            gshape = tuple(data.shape)
            split = sanitize_axis(gshape, split)
            _, _, sl = comm.chunk(gshape, split)
            local = torch.tensor(np.asarray(data[sl]), dtype=htype.torch_type(), device=device.torch_device)
        return DNDarray(local, gshape, htype, split, device, comm, True)

    def save_netcdf(data: DNDarray, path: str, variable: str, mode: str = "w", dimension_names=None,
                    **kwargs) -> None:
        comm = data.comm
        if dimension_names is None:
            dimension_names = ["dim_{}".format(i) for i in range(data.ndim)]
        exc = None
        if comm.rank == 0:
            try:
                with nc.Dataset(path, mode) as handle:
                    for name, size in zip(dimension_names, data.gshape):
                        if name not in handle.dimensions:
                            handle.createDimension(name, size)
                    handle.createVariable(variable, data.larray.cpu().numpy().dtype, tuple(dimension_names), **kwargs)
            except Exception as e:
                exc = e
        _exception_barrier(comm, exc)
        counts, displs = data.counts_displs() if data.is_distributed() else ((data.gshape[0],), (0,))
        for r in range(comm.size):
            if r == comm.rank and (data.is_distributed() or r == 0):
                with nc.Dataset(path, "r+") as handle:
                    sl = [slice(None)] * data.ndim
                    if data.is_distributed():
                        sl[data.split] = slice(displs[r], displs[r] + counts[r])
                    handle[variable][tuple(sl)] = data.larray.cpu().numpy()
            comm.Barrier()

    DNDarray.save_netcdf = lambda self, path, variable, mode="w", **kwargs: save_netcdf(self, path, variable, mode, **kwargs)


# --------------------------------------------------------------------------------------------- dispatch
def load(path: str, *args, **kwargs) -> DNDarray:
    """Load by file extension: .h5/.hdf5, .nc/.nc4/.netcdf, .csv, .npy."""
    if not isinstance(path, str):
        raise TypeError("Expected path to be str, but was {}".format(type(path)))
    ext = os.path.splitext(path)[-1].strip().lower()
    if ext in (".h5", ".hdf5"):
        if supports_hdf5():
            return load_hdf5(path, *args, **kwargs)
        raise RuntimeError("hdf5 is required for file extension {}".format(ext))
    if ext in (".nc", ".nc4", ".netcdf"):
        if supports_netcdf():
            return load_netcdf(path, *args, **kwargs)
        raise RuntimeError("netcdf is required for file extension {}".format(ext))
    if ext == ".csv":
        return load_csv(path, *args, **kwargs)
    if ext == ".npy":
        return load_npy(path, *args, **kwargs)
    raise ValueError("Unsupported file extension {}".format(ext))


def save(data: DNDarray, path: str, *args, **kwargs) -> None:
    """Save by file extension: .h5/.hdf5, .nc/.nc4/.netcdf, .csv, .npy."""
    if not isinstance(path, str):
        raise TypeError("Expected path to be str, but was {}".format(type(path)))
    ext = os.path.splitext(path)[-1].strip().lower()
    if ext in (".h5", ".hdf5"):
        if supports_hdf5():
            return save_hdf5(data, path, *args, **kwargs)
        raise RuntimeError("hdf5 is required for file extension {}".format(ext))
    if ext in (".nc", ".nc4", ".netcdf"):
        if supports_netcdf():
            return save_netcdf(data, path, *args, **kwargs)
        raise RuntimeError("netcdf is required for file extension {}".format(ext))
    if ext == ".csv":
        return save_csv(data, path, *args, **kwargs)
    if ext == ".npy":
        return save_npy(data, path)
    raise ValueError("Unsupported file extension {}".format(ext))


DNDarray.save = lambda self, path, *args, **kwargs: save(self, path, *args, **kwargs)
