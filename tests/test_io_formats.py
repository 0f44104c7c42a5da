"""File-format details of the dependency-free IO fallbacks (no GPU, one process)."""
import os
import struct

import numpy as np
import pytest

from heat_amd.core import _h5lite, _ncclassic


def _fletcher32_wordwise(data: bytes) -> int:
    """Word-by-word transcription of HDF5's H5_checksum_fletcher32 (uint32 sums)."""
    n = len(data) // 2
    s1 = s2 = 0
    i = 0
    while n:
        t = min(n, 360)
        n -= t
        for _ in range(t):
            s1 = (s1 + ((data[i] << 8) | data[i + 1])) & 0xFFFFFFFF
            i += 2
            s2 = (s2 + s1) & 0xFFFFFFFF
        s1 = (s1 & 0xFFFF) + (s1 >> 16)
        s2 = (s2 & 0xFFFF) + (s2 >> 16)
    if len(data) % 2:
        s1 += data[i] << 8
        s2 += s1
        s1 = (s1 & 0xFFFF) + (s1 >> 16)
        s2 = (s2 & 0xFFFF) + (s2 >> 16)
    s1 = (s1 & 0xFFFF) + (s1 >> 16)
    s2 = (s2 & 0xFFFF) + (s2 >> 16)
    return (s2 << 16) | s1


def test_fletcher32_all_ones_chunk():
    # HDF5 gives 0xffffffff here; a "% 65535" reduction gives 0 and HDF5 refuses the chunk
    assert _h5lite._fletcher32(b"\xff" * 4096) == 0xFFFFFFFF
    assert _h5lite._fletcher32(b"\xff" * 4097) == _fletcher32_wordwise(b"\xff" * 4097)


@pytest.mark.parametrize("n", [1, 2, 3, 719, 720, 721, 5000, 65535])
def test_fletcher32_matches_wordwise(n):
    rng = np.random.default_rng(n)
    data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    assert _h5lite._fletcher32(data) == _fletcher32_wordwise(data)


def test_fletcher32_verified_on_read(tmp_path):
    import heat_amd as ht

    a = np.full((64, 16), -1, dtype=np.int32)   # all-0xFF chunks
    p = str(tmp_path / "f.h5")
    ht.save_hdf5(ht.array(a, split=0), p, "d", chunks=(16, 16), fletcher32=True)
    assert np.array_equal(ht.load_hdf5(p, "d", dtype=ht.int32).numpy(), a)
    # corrupt one data byte of the first chunk: the read must fail, not return garbage
    raw = bytearray(open(p, "rb").read())
    pos = raw.find(b"\xff" * 64)
    raw[pos] = 0x00
    open(p, "wb").write(bytes(raw))
    with pytest.raises(IOError):
        ht.load_hdf5(p, "d", dtype=ht.int32).numpy()


def test_fletcher32_accepts_reversed_and_legacy_forms():
    """HDF5 reads chunks whose checksum is byte-pair swapped (libraries before 1.6.3); this
    package's pre-round-4 writer folded with % 65535; a wrong checksum is still refused."""
    rng = np.random.default_rng(5)
    body = rng.integers(0, 256, 1000, dtype=np.uint8).tobytes()
    c = _h5lite._fletcher32(body)
    rev = ((c & 0x00FF00FF) << 8) | ((c >> 8) & 0x00FF00FF)
    assert _h5lite._fletcher32_ok(body, c) and _h5lite._fletcher32_ok(body, rev)
    assert not _h5lite._fletcher32_ok(body, c ^ 0x10)
    ones = b"\xff" * 4096                      # sums are multiples of 65535: the two folds differ
    assert _h5lite._fletcher32(ones) == 0xFFFFFFFF and _h5lite._fletcher32(ones, legacy_mod=True) == 0
    assert _h5lite._fletcher32_ok(ones, 0)


def test_netcdf_cdf5_header_roundtrip(tmp_path):
    p = str(tmp_path / "x.nc")
    h = _ncclassic.write_with_variable(p, None, "v", ["a", "b"], (3, 4), _ncclassic.nc_type_for(np.int64), False)
    assert h.version == 5
    h2 = _ncclassic.parse(p)
    assert h2.version == 5 and h2.dims == [("a", 3), ("b", 4)] and h2.vars[0].nc_type == 10
    shape, dt, begin, rec = _ncclassic.layout(h2, "v")
    assert shape == (3, 4) and dt == np.dtype(">i8") and rec is None
    assert os.path.getsize(p) == begin + 3 * 4 * 8
    # a record variable added next to it; the fixed variable's data moves with the rewrite
    mm = _ncclassic.memmap(p, shape, dt, begin, rec)
    mm[:] = np.arange(12).reshape(3, 4) * 2 ** 40
    mm.flush()
    del mm
    h3 = _ncclassic.write_with_variable(p, h2, "r", ["t", "b"], (0, 4), _ncclassic.nc_type_for(np.uint8), True)
    h3 = _ncclassic.grow_records(p, h3, 5)
    shape, dt, begin, rec = _ncclassic.layout(_ncclassic.parse(p), "v")
    assert np.array_equal(np.asarray(_ncclassic.memmap(p, shape, dt, begin, rec, mode="r")),
                          np.arange(12).reshape(3, 4) * 2 ** 40)
    shape, dt, begin, rec = _ncclassic.layout(_ncclassic.parse(p), "r")
    assert shape == (5, 4) and dt == np.dtype("u1") and rec == 4


def test_netcdf_classic_v2_readable_by_scipy(tmp_path):
    from scipy.io import netcdf_file

    p = str(tmp_path / "c.nc")
    h = _ncclassic.write_with_variable(p, None, "v", ["a"], (5,), _ncclassic.nc_type_for(np.float32), False)
    shape, dt, begin, rec = _ncclassic.layout(h, "v")
    mm = _ncclassic.memmap(p, shape, dt, begin, rec)
    mm[:] = np.arange(5, dtype=np.float32)
    mm.flush()
    del mm
    with netcdf_file(p, "r", mmap=False) as f:
        assert np.array_equal(f.variables["v"].data, np.arange(5, dtype=np.float32))
