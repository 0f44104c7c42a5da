"""
Classic netCDF files without the netCDF C library: CDF-1 (32-bit offsets), CDF-2 (64-bit
offsets) and CDF-5 (64-bit data: ``NC_UBYTE``, ``NC_USHORT``, ``NC_UINT``, ``NC_INT64``,
``NC_UINT64`` and 64-bit sizes).

The reference writes through ``netCDF4.Dataset`` (``heat/core/io.py:573, 599``); that package is
not importable in this image. This module is the fallback used by ``heat_amd.core.io``: it parses
a header, computes a variable's data layout (fixed-size variables are one contiguous block,
record variables are strided by the record size), and re-writes a file with an added dimension /
variable, copying the data of the variables already present. The data itself is then written
in place by every rank through a memory map, in parallel.

A file is written as CDF-2 unless a variable needs a CDF-5 type, in which case the whole file
becomes CDF-5: int64 / uint8 / uint16 / uint32 / uint64 / bool data is stored LOSSLESSLY (bool as
``NC_UBYTE`` 0/1, float16 as ``NC_FLOAT``); complex data raises ``TypeError``. Byte-level parity
with files written by the netCDF C library is unpinned (that library is absent here); the layout
follows the published classic / CDF-5 format specification.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

__all__ = ["Header", "Var", "parse", "layout", "nc_type_for", "write_with_variable", "memmap"]

# nc_type -> big-endian numpy dtype
NC_DTYPES = {1: np.dtype("i1"), 2: np.dtype("S1"), 3: np.dtype(">i2"), 4: np.dtype(">i4"), 5: np.dtype(">f4"),
             6: np.dtype(">f8"), 7: np.dtype("u1"), 8: np.dtype(">u2"), 9: np.dtype(">u4"), 10: np.dtype(">i8"),
             11: np.dtype(">u8")}
_CDF5_ONLY = {7, 8, 9, 10, 11}
_NC_DIMENSION, _NC_VARIABLE, _NC_ATTRIBUTE = 0x0A, 0x0B, 0x0C


def nc_type_for(np_dtype) -> int:
    """nc_type storing ``np_dtype`` without loss (bool -> NC_UBYTE, float16 -> NC_FLOAT)."""
    dt = np.dtype(np_dtype)
    if dt == np.bool_:
        return 7
    if dt.kind == "f" and dt.itemsize == 2:
        return 5
    if dt.kind == "S" and dt.itemsize == 1:
        return 2
    table = {("i", 1): 1, ("i", 2): 3, ("i", 4): 4, ("i", 8): 10, ("u", 1): 7, ("u", 2): 8, ("u", 4): 9,
             ("u", 8): 11, ("f", 4): 5, ("f", 8): 6}
    key = (dt.kind, dt.itemsize)
    if key not in table:
        raise TypeError("netCDF has no type for {}".format(dt))
    return table[key]


@dataclass
class Var:
    name: str
    dimids: List[int]
    nc_type: int
    atts: list = field(default_factory=list)  # [(name, nc_type, count, raw bytes incl. padding)]
    vsize: int = 0
    begin: int = 0


@dataclass
class Header:
    version: int = 2
    numrecs: int = 0
    dims: List[Tuple[str, int]] = field(default_factory=list)  # length 0 = the record dimension
    gatts: list = field(default_factory=list)
    vars: List[Var] = field(default_factory=list)

    def var(self, name: str) -> Optional[Var]:
        for v in self.vars:
            if v.name == name:
                return v
        return None

    def is_record(self, v: Var) -> bool:
        return bool(v.dimids) and self.dims[v.dimids[0]][1] == 0

    def shape(self, v: Var) -> tuple:
        return tuple(self.numrecs if (k == 0 and self.is_record(v)) else self.dims[d][1]
                     for k, d in enumerate(v.dimids))

    def record_size(self) -> int:
        rec = [v for v in self.vars if self.is_record(v)]
        if len(rec) == 1:  # a single record variable is not padded per record
            v = rec[0]
            return int(np.prod(self.shape(v)[1:], dtype=np.int64)) * NC_DTYPES[v.nc_type].itemsize
        return sum(v.vsize for v in rec)


# ------------------------------------------------------------------------------------------ parse
def parse(path: str) -> Header:
    """Read the header of a CDF-1 / CDF-2 / CDF-5 file."""
    with open(path, "rb") as f:
        buf = bytearray(f.read(1 << 16))
        pos = 0

        def need(n):
            nonlocal buf
            while pos + n > len(buf):
                more = f.read(max(1 << 16, n))
                if not more:
                    raise ValueError("truncated netCDF header in {}".format(path))
                buf += more

        def i4():
            nonlocal pos
            need(4)
            v = struct.unpack_from(">i", buf, pos)[0]
            pos += 4
            return v

        def i8():
            nonlocal pos
            need(8)
            v = struct.unpack_from(">q", buf, pos)[0]
            pos += 8
            return v

        need(4)
        if bytes(buf[:3]) != b"CDF" or buf[3] not in (1, 2, 5):
            raise ValueError("{} is not a classic netCDF file".format(path))
        version = buf[3]
        nn = i8 if version == 5 else i4  # NON_NEG width

        def name():
            nonlocal pos
            n = nn()
            need(n + (-n) % 4)
            v = bytes(buf[pos: pos + n]).decode("utf-8")
            pos += n + (-n) % 4
            return v

        def atts():
            nonlocal pos
            tag, n = i4(), nn()
            out = []
            for _ in range(n if tag else 0):
                an = name()
                t, cnt = i4(), nn()
                size = cnt * NC_DTYPES[t].itemsize
                size += (-size) % 4
                need(size)
                out.append((an, t, cnt, bytes(buf[pos: pos + size])))
                pos += size
            return out

        pos = 4
        h = Header(version=version)
        h.numrecs = nn()
        tag, nd = i4(), nn()
        h.dims = [(name(), nn()) for _ in range(nd if tag else 0)]
        h.gatts = atts()
        tag, nv = i4(), nn()
        for _ in range(nv if tag else 0):
            vn = name()
            ndv = nn()
            dimids = [nn() for _ in range(ndv)]
            va = atts()
            t, vsize = i4(), nn()
            begin = i4() if version == 1 else i8()
            h.vars.append(Var(vn, dimids, t, va, vsize, begin))
    return h


def layout(h: Header, variable: str):
    """(shape, big-endian dtype, begin offset, record stride in bytes or None)."""
    v = h.var(variable)
    if v is None:
        raise KeyError(variable)
    return h.shape(v), NC_DTYPES[v.nc_type], v.begin, (h.record_size() if h.is_record(v) else None)


def memmap(path: str, shape, dtype, begin: int, recsize: Optional[int], mode: str = "r+"):
    """Memory map of a variable's data (a record variable as a strided view)."""
    if recsize is None:
        if int(np.prod(shape, dtype=np.int64)) == 0:
            return np.zeros(shape, dtype=dtype)
        return np.memmap(path, dtype=dtype, mode=mode, offset=begin, shape=tuple(shape))
    nrec = shape[0]
    inner = int(np.prod(shape[1:], dtype=np.int64)) if len(shape) > 1 else 1
    if nrec == 0 or inner == 0:
        return np.zeros(shape, dtype=dtype)
    raw = np.memmap(path, dtype=np.uint8, mode=mode, offset=begin,
                    shape=((nrec - 1) * recsize + inner * dtype.itemsize,))
    strides = (recsize,) + tuple(int(np.prod(shape[k + 1:], dtype=np.int64)) * dtype.itemsize
                                 for k in range(1, len(shape)))
    return np.ndarray(tuple(shape), dtype=dtype, buffer=raw, strides=strides)


# ------------------------------------------------------------------------------------------ write
def _encode(h: Header) -> bytes:
    v5 = h.version == 5
    nn = (lambda x: struct.pack(">q", x)) if v5 else (lambda x: struct.pack(">i", x))

    def name(s: str) -> bytes:
        raw = s.encode("utf-8")
        return nn(len(raw)) + raw + b"\0" * ((-len(raw)) % 4)

    def atts(lst) -> bytes:
        if not lst:
            return struct.pack(">i", 0) + nn(0)
        return struct.pack(">i", _NC_ATTRIBUTE) + nn(len(lst)) + b"".join(
            name(an) + struct.pack(">i", t) + nn(cnt) + raw for an, t, cnt, raw in lst)

    out = [b"CDF" + bytes([h.version]), nn(h.numrecs)]
    out.append(struct.pack(">i", _NC_DIMENSION if h.dims else 0) + nn(len(h.dims)))
    out += [name(dn) + nn(dl) for dn, dl in h.dims]
    out.append(atts(h.gatts))
    out.append(struct.pack(">i", _NC_VARIABLE if h.vars else 0) + nn(len(h.vars)))
    for v in h.vars:
        vs = v.vsize if v5 else min(v.vsize, 2 ** 32 - 4)
        if not v5 and vs >= 2 ** 31:
            vs = 2 ** 32 - 1  # netCDF convention for a too-large last variable (read as unsigned)
            vs = struct.unpack(">i", struct.pack(">I", vs))[0]
        out.append(name(v.name) + nn(len(v.dimids)) + b"".join(nn(d) for d in v.dimids) + atts(v.atts)
                   + struct.pack(">i", v.nc_type) + nn(vs)
                   + (struct.pack(">i", v.begin) if h.version == 1 else struct.pack(">q", v.begin)))
    return b"".join(out)


def _assign_offsets(h: Header) -> int:
    """Set vsize / begin of every variable (fixed variables after the header in order, then the
    record section); returns the file size."""
    for v in h.vars:
        inner = [h.dims[d][1] for k, d in enumerate(v.dimids) if not (k == 0 and h.is_record(v))]
        n = int(np.prod(inner, dtype=np.int64)) * NC_DTYPES[v.nc_type].itemsize
        v.vsize = n + (-n) % 4
    pos = len(_encode(h))  # begin fields have a fixed width: the header size does not depend on them
    for v in h.vars:
        if not h.is_record(v):
            v.begin = pos
            pos += v.vsize
    rec0 = pos
    for v in h.vars:
        if h.is_record(v):
            v.begin = pos
            pos += v.vsize
    return rec0 + h.numrecs * h.record_size()


def _copy(src, dst, s_off: int, d_off: int, n: int) -> None:
    src.seek(s_off)
    dst.seek(d_off)
    while n > 0:
        chunk = src.read(min(n, 64 << 20))
        if not chunk:
            break
        dst.write(chunk)
        n -= len(chunk)


def write_with_variable(path: str, old: Optional[Header], variable: str, dims: List[str], gshape,
                        nc_type: int, unlimited: bool, numrecs: int = 0) -> Header:
    """Write ``path`` holding everything of ``old`` (None: a new file) plus ``variable`` with
    dimensions ``dims`` of lengths ``gshape`` (the first one unlimited if ``unlimited``); the new
    variable's data is zero. Existing data is copied into the new layout; the file is replaced
    atomically. Returns the new header."""
    h = Header(version=old.version if old is not None else 2, numrecs=old.numrecs if old is not None else 0,
               dims=list(old.dims) if old is not None else [], gatts=list(old.gatts) if old is not None else [],
               vars=[Var(v.name, list(v.dimids), v.nc_type, list(v.atts), v.vsize, v.begin)
                     for v in old.vars] if old is not None else [])
    if h.var(variable) is not None:
        raise ValueError("variable {!r} already exists".format(variable))
    dimids = []
    for i, (dn, size) in enumerate(zip(dims, gshape)):
        want = 0 if (unlimited and i == 0) else int(size)
        ids = [k for k, (n, _) in enumerate(h.dims) if n == dn]
        if ids:
            have = h.dims[ids[0]][1]
            if have != want and not (have == 0 and i == 0):
                raise ValueError("dimension {!r} has length {} in the file, the data needs {}".format(
                    dn, have or "UNLIMITED", want or "UNLIMITED"))
            dimids.append(ids[0])
        else:
            if want == 0 and any(l == 0 for _, l in h.dims):
                raise ValueError("a classic netCDF file has at most one unlimited dimension")
            h.dims.append((dn, want))
            dimids.append(len(h.dims) - 1)
    if any(h.dims[d][1] == 0 for d in dimids[1:]):
        raise ValueError("the unlimited dimension must be the first dimension of a variable")
    h.vars.append(Var(variable, dimids, nc_type))
    if nc_type in _CDF5_ONLY or any(v.nc_type in _CDF5_ONLY for v in h.vars):
        h.version = 5
    if h.is_record(h.vars[-1]):
        h.numrecs = max(h.numrecs, int(numrecs))
    size = _assign_offsets(h)
    tmp = path + ".heat_tmp"
    with open(tmp, "wb") as dst:
        dst.write(_encode(h))
        if old is not None:
            with open(path, "rb") as src:
                rec_old, rec_new = old.record_size(), h.record_size()
                for ov in old.vars:
                    nv = h.var(ov.name)
                    if not old.is_record(ov):
                        n = int(np.prod(old.shape(ov), dtype=np.int64)) * NC_DTYPES[ov.nc_type].itemsize
                        _copy(src, dst, ov.begin, nv.begin, n)
                    else:
                        n = int(np.prod(old.shape(ov)[1:], dtype=np.int64)) * NC_DTYPES[ov.nc_type].itemsize
                        for r in range(old.numrecs):
                            _copy(src, dst, ov.begin + r * rec_old, nv.begin + r * rec_new, n)
        dst.truncate(size + (-size) % 4)
    os.replace(tmp, path)
    return h


def grow_records(path: str, h: Header, numrecs: int) -> Header:
    """Raise the record count to ``numrecs`` (new records are zero)."""
    if numrecs <= h.numrecs:
        return h
    h.numrecs = int(numrecs)
    with open(path, "r+b") as f:
        f.seek(4)
        f.write(struct.pack(">q", h.numrecs) if h.version == 5 else struct.pack(">i", h.numrecs))
        rec0 = min((v.begin for v in h.vars if h.is_record(v)), default=0)
        end = rec0 + h.numrecs * h.record_size()
        f.seek(0, 2)
        if f.tell() < end:
            f.truncate(end + (-end) % 4)
    return h
