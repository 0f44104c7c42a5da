"""
Parallel IO (reference ``heat/core/io.py``: ``load_hdf5`` 55, ``save_hdf5`` 147, ``load_netcdf`` 265,
``save_netcdf`` 348, ``load`` 659, ``load_csv`` 710, ``save`` 923).

* HDF5 / NetCDF: through ``h5py`` / ``netCDF4`` when importable, otherwise through the built-in
  dependency-free HDF5 reader/writer (``_h5lite``) and classic netCDF files (same layout as the
  reference; every rank reads only its hyperslab and writes its slab in place, in parallel).
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
from . import _h5lite
from .stride_tricks import sanitize_axis

__all__ = ["load", "load_csv", "save", "save_csv", "load_npy", "save_npy", "supports_hdf5", "supports_netcdf",
           "load_hdf5", "save_hdf5", "load_netcdf", "save_netcdf"]

try:
    import h5py  # noqa: F401
except ImportError:
    h5py = None
try:
    import netCDF4 as nc  # noqa: F401
except ImportError:
    nc = None


def supports_hdf5() -> bool:
    """HDF5 is always available (h5py, or the built-in reader/writer ``_h5lite``)."""
    return True


def supports_netcdf() -> bool:
    """netCDF is always available (netCDF4, or netCDF-4/HDF5 reading via ``_h5lite`` and classic
    netCDF reading (scipy) / writing (built in))."""
    return True


def _exception_barrier(comm, exc: Optional[BaseException]):
    """Propagate a failure on any rank to every rank (reference io.py:593-650, made generic)."""
    from ..parallel.guard import exception_barrier

    exception_barrier(comm, exc)


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
def _hyperslab(gshape, split, comm):
    _, _, sl = comm.chunk(tuple(gshape), split)
    return sl


def load_hdf5(path: str, dataset: str, dtype=types.float32, load_fraction: float = 1.0,
              split: Optional[int] = None, device=None, comm=None) -> DNDarray:
    """Load an HDF5 dataset; every rank reads only its hyperslab (h5py when installed, otherwise
    the built-in reader ``_h5lite``, which memory-maps contiguous storage)."""
    if not isinstance(path, str):
        raise TypeError("path must be str, not {}".format(type(path)))
    if not isinstance(dataset, str):
        raise TypeError("dataset must be str, not {}".format(type(dataset)))
    if not isinstance(load_fraction, float):
        raise TypeError("load_fraction must be float, but is {}".format(type(load_fraction)))
    if load_fraction <= 0.0 or load_fraction > 1.0:
        raise ValueError("load_fraction must be between 0 (exclusive) and 1 (inclusive), not {}".format(load_fraction))
    comm = sanitize_comm(comm)
    device = devices.sanitize_device(device)
    htype = types.canonical_heat_type(dtype)
    handle = h5py.File(path, "r") if h5py is not None else _h5lite.open_file(path)
    try:
        data = handle[dataset]
        gshape = list(data.shape)
        if split is not None:
            split = sanitize_axis(tuple(gshape), split)
            gshape[split] = int(gshape[split] * load_fraction)
        gshape = tuple(gshape)
        split = sanitize_axis(gshape, split)
        local = np.asarray(data[_hyperslab(gshape, split, comm)])
    finally:
        handle.close()
    t = torch.from_numpy(np.ascontiguousarray(local).astype(local.dtype.newbyteorder("=")))
    t = t.to(device=device.torch_device, dtype=htype.torch_type())
    return DNDarray(t, gshape, htype, split, device, comm, True)


def save_hdf5(data: DNDarray, path: str, dataset: str, mode: str = "w", **kwargs) -> None:
    """Write a DNDarray into an HDF5 dataset. Without h5py (built-in writer) rank 0 declares the
    dataset and every rank then writes its slab into the pre-allocated storage in parallel."""
    if not isinstance(data, DNDarray):
        raise TypeError("data must be heat tensor, not {}".format(type(data)))
    if not isinstance(path, str):
        raise TypeError("path must be str, not {}".format(type(path)))
    if not isinstance(dataset, str):
        raise TypeError("dataset must be str, not {}".format(type(path)))
    if mode not in ("w", "a", "r+"):
        raise ValueError("mode was {}, not in possible modes ['w', 'a', 'r+']".format(mode))
    comm = data.comm
    np_dtype = np.dtype(torch.empty(0, dtype=data.larray.dtype).numpy().dtype)
    counts, displs = data.counts_displs() if data.is_distributed() else ((None,), (None,))
    exc = None
    if comm.rank == 0:
        try:
            if h5py is not None:
                with h5py.File(path, mode) as handle:
                    handle.create_dataset(dataset, data.gshape, dtype=np_dtype, **kwargs)
            else:
                if mode == "w" or not os.path.exists(path):
                    _h5lite.create_file(path)
                _h5lite.create_dataset(path, dataset, data.gshape, np_dtype)
        except Exception as e:  # propagated to every rank
            exc = e
    _exception_barrier(comm, exc)
    local = data.larray.cpu().numpy()
    if not data.is_distributed():
        if comm.rank == 0:
            _write_slab(path, dataset, (slice(None),) * data.ndim, local)
        comm.Barrier()
        return
    me = comm.rank
    sl = [slice(None)] * data.ndim
    sl[data.split] = slice(displs[me], displs[me] + counts[me])
    if h5py is not None:  # h5py without MPI-IO: one writer at a time
        for r in range(comm.size):
            if r == me and counts[me]:
                _write_slab(path, dataset, tuple(sl), local)
            comm.Barrier()
    else:
        if counts[me]:
            _write_slab(path, dataset, tuple(sl), local)
        comm.Barrier()


def _write_slab(path: str, dataset: str, sl, local: np.ndarray) -> None:
    if h5py is not None:
        with h5py.File(path, "r+") as handle:
            handle[dataset][sl] = local
        return
    mm = _h5lite.open_for_write(path, dataset)
    mm[sl] = local.astype(mm.dtype, copy=False)
    mm.flush()
    del mm


DNDarray.save_hdf5 = lambda self, path, dataset, mode="w", **kwargs: save_hdf5(self, path, dataset, mode, **kwargs)


# --------------------------------------------------------------------------------------------- netcdf
def _netcdf3_header(variable: str, dims: List[str], shape, np_dtype: np.dtype) -> Tuple[bytes, int]:
    """Classic netCDF (CDF-2, 64-bit offsets) header for ONE fixed-size variable; returns
    (header bytes, data offset). Layout: magic, numrecs, dim_list, gatt_list, var_list."""
    import struct

    codes = {np.dtype("i1"): 1, np.dtype("S1"): 2, np.dtype("i2"): 3, np.dtype("i4"): 4, np.dtype("f4"): 5,
             np.dtype("f8"): 6}
    if np_dtype not in codes:
        raise TypeError("netCDF classic has no {}".format(np_dtype))

    def name(n: str) -> bytes:
        raw = n.encode("utf-8")
        return struct.pack(">i", len(raw)) + raw + b"\0" * ((-len(raw)) % 4)

    h = b"CDF\x02" + struct.pack(">i", 0)
    h += struct.pack(">ii", 0x0A, len(dims)) + b"".join(name(d) + struct.pack(">i", int(s)) for d, s in zip(dims, shape))
    h += struct.pack(">ii", 0, 0)
    vsize = int(np.prod(shape)) * np_dtype.itemsize
    var = name(variable) + struct.pack(">i", len(dims)) + b"".join(struct.pack(">i", i) for i in range(len(dims)))
    var += struct.pack(">ii", 0, 0) + struct.pack(">ii", codes[np_dtype], min(vsize + ((-vsize) % 4), 2 ** 31 - 1))
    begin = len(h) + 8 + len(var) + 8
    h += struct.pack(">ii", 0x0B, 1) + var + struct.pack(">q", begin)
    assert len(h) == begin
    return h, begin


def load_netcdf(path: str, variable: str, dtype=types.float32, split: Optional[int] = None, device=None,
                comm=None) -> DNDarray:
    """Load a netCDF variable (netCDF4 when installed; otherwise netCDF-4/HDF5 files through the
    built-in HDF5 reader and classic files through ``scipy.io.netcdf_file``)."""
    if not isinstance(path, str):
        raise TypeError("path must be str, not {}".format(type(path)))
    if not isinstance(variable, str):
        raise TypeError("dataset must be str, not {}".format(type(variable)))
    comm = sanitize_comm(comm)
    device = devices.sanitize_device(device)
    htype = types.canonical_heat_type(dtype)
    if nc is not None:
        with nc.Dataset(path, "r") as handle:
            data = handle[variable]
            gshape = tuple(data.shape)
            split = sanitize_axis(gshape, split)
            local = np.asarray(data[_hyperslab(gshape, split, comm)])
    elif _h5lite.is_hdf5(path):
        with _h5lite.open_file(path) as handle:
            data = handle[variable]
            gshape = tuple(data.shape)
            split = sanitize_axis(gshape, split)
            local = np.asarray(data[_hyperslab(gshape, split, comm)])
    else:
        from scipy.io import netcdf_file

        with netcdf_file(path, "r", mmap=True) as handle:
            data = handle.variables[variable].data
            gshape = tuple(data.shape)
            split = sanitize_axis(gshape, split)
            local = np.array(data[_hyperslab(gshape, split, comm)])
            del data  # the mmap must not be referenced when the file closes
    t = torch.from_numpy(np.ascontiguousarray(local).astype(local.dtype.newbyteorder("=")))
    t = t.to(device=device.torch_device, dtype=htype.torch_type())
    return DNDarray(t, gshape, htype, split, device, comm, True)


def save_netcdf(data: DNDarray, path: str, variable: str, mode: str = "w", dimension_names=None,
                **kwargs) -> None:
    """Write a DNDarray as a netCDF variable. Without netCDF4 a classic (CDF-2) file is written:
    rank 0 writes the header, every rank writes its slab of the big-endian data block in place."""
    if not isinstance(data, DNDarray):
        raise TypeError("data must be heat tensor, not {}".format(type(data)))
    if not isinstance(path, str):
        raise TypeError("path must be str, not {}".format(type(path)))
    if not isinstance(variable, str):
        raise TypeError("variable must be str, not {}".format(type(variable)))
    comm = data.comm
    if dimension_names is None:
        dimension_names = ["dim_{}".format(i) for i in range(data.ndim)]
    elif isinstance(dimension_names, str):
        dimension_names = [dimension_names]
    if len(dimension_names) != data.ndim:
        raise ValueError("{0} names given for {1} dimensions".format(len(dimension_names), data.ndim))
    counts, displs = data.counts_displs() if data.is_distributed() else ((data.gshape[0] if data.ndim else 1,), (0,))
    local = data.larray.cpu().numpy()
    sl = [slice(None)] * data.ndim
    if data.is_distributed():
        sl[data.split] = slice(displs[comm.rank], displs[comm.rank] + counts[comm.rank])
    exc = None
    if nc is not None:
        if comm.rank == 0:
            try:
                with nc.Dataset(path, mode) as handle:
                    for name, size in zip(dimension_names, data.gshape):
                        if name not in handle.dimensions:
                            handle.createDimension(name, size)
                    handle.createVariable(variable, local.dtype, tuple(dimension_names), **kwargs)
            except Exception as e:
                exc = e
        _exception_barrier(comm, exc)
        for r in range(comm.size):
            if r == comm.rank and (data.is_distributed() or r == 0):
                with nc.Dataset(path, "r+") as handle:
                    handle[variable][tuple(sl)] = local
            comm.Barrier()
        return
    if mode != "w":
        raise NotImplementedError("without netCDF4 only mode='w' (a new classic file) is supported")
    np_dtype = np.dtype(local.dtype)
    if np_dtype == np.dtype("i8"):
        np_dtype = np.dtype("i4")
    elif np_dtype == np.dtype("bool") or np_dtype == np.dtype("u1"):
        np_dtype = np.dtype("i1")
    begin = 0
    if comm.rank == 0:
        try:
            header, begin = _netcdf3_header(variable, dimension_names, data.gshape, np_dtype)
            nbytes = int(np.prod(data.gshape)) * np_dtype.itemsize
            with open(path, "wb") as f:
                f.write(header)
                f.truncate(begin + nbytes + ((-nbytes) % 4))
        except Exception as e:
            exc = e
    _exception_barrier(comm, exc)
    begin = comm.bcast(begin, root=0)
    if data.is_distributed() or comm.rank == 0:
        if local.size:
            mm = np.memmap(path, dtype=np_dtype.newbyteorder(">"), mode="r+", offset=begin, shape=data.gshape)
            mm[tuple(sl)] = local.astype(np_dtype)
            mm.flush()
            del mm
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
