"""Parity with ``heat/core/tests/test_io.py``: load/save dispatch by extension, CSV (headers,
split, per-rank byte ranges), HDF5 and netCDF round trips on every split (modes, slices, unlimited
dimensions) and the reference's exceptions. The reference's own fixtures (``iris.csv``/``.h5``/``.nc``,
plain data files) are read when present - they hold the same 150 x 4 iris table."""
import os
import tempfile

import numpy as np
import torch

import heat_amd as ht

from ._util import close, raises, same, splits

DS = "/root/reference/heat/datasets"
CSV, H5, NC = os.path.join(DS, "iris.csv"), os.path.join(DS, "iris.h5"), os.path.join(DS, "iris.nc")


def _tmp(name):
    # one path for all ranks of the job (same host): rank 0's pid keys it
    d = os.path.join(tempfile.gettempdir(), "heat_amd_io_{}".format(os.environ.get("MASTER_PORT", os.getpid())))
    if ht.MPI_WORLD.rank == 0:
        os.makedirs(d, exist_ok=True)
    ht.MPI_WORLD.Barrier()
    return os.path.join(d, name)


def _iris_np():
    if os.path.exists(CSV):
        return np.loadtxt(CSV, delimiter=";").astype(np.float32)
    return None


def test_load():
    ref = _iris_np()
    if ref is None:
        return
    for split in (None, 0, 1):
        a = ht.load(H5, dataset="data", split=split)
        assert a.shape == (150, 4) and a.dtype == ht.float32 and a.split == split
        close(a, ref, atol=1e-6)
        b = ht.load(NC, variable="data", split=split)
        close(b, ref, atol=1e-6)
        c = ht.load(CSV, sep=";", split=split)
        close(c, ref, atol=1e-6)


def test_load_csv():
    ref = _iris_np()
    if ref is None:
        return
    a = ht.load_csv(CSV, sep=";")
    assert len(a) == 150 and a.shape == (150, 4)
    assert torch.equal(a.larray[0].cpu(), torch.tensor([5.1, 3.5, 1.4, 0.2]))
    assert torch.equal(a.larray[9].cpu(), torch.tensor([4.9, 3.1, 1.5, 0.1]))
    a = ht.load_csv(CSV, sep=";", split=0)
    counts, _, _ = a.comm.counts_displs_shape((150, 4), 0)
    assert a.gshape == (150, 4) and a.lshape == (counts[a.comm.rank], 4)
    same(a, ref)
    a = ht.load_csv(CSV, sep=";", header_lines=9, dtype=ht.float32, split=0)
    counts, _, _ = a.comm.counts_displs_shape((141, 4), 0)
    assert a.gshape == (141, 4) and a.lshape == (counts[a.comm.rank], 4) and a.dtype == ht.float32
    same(a, ref[9:])
    a = ht.load_csv(CSV, sep=";", split=1)
    assert a.shape == (150, 4) and a.lshape[0] == 150
    assert ht.equal(ht.load_csv(CSV, sep=";", split=0), ht.load(CSV, sep=";", split=0))
    a = ht.load_csv(CSV, sep=";", header_lines=100, split=0)
    assert a.shape == (50, 4)
    same(a, ref[100:])
    raises(TypeError, ht.load_csv, 12314)
    raises(TypeError, ht.load_csv, CSV, sep=11)
    raises(TypeError, ht.load_csv, CSV, header_lines="3", sep=";", split=0)


def test_load_exception():
    raises(IOError, ht.load, "foo.h5", "data")
    raises(IOError, ht.load, "foo.nc", "data")
    raises(ValueError, ht.load, "iris.json", "data")
    raises(ValueError, ht.load, "iris", "data")


def test_save():
    x = np.arange(7 * 5 * 3, dtype=np.float32).reshape(7, 5, 3)
    for ext, kw, loadkw in ((".h5", {"dataset": "data"}, {"dataset": "data"}),
                            (".nc", {"variable": "data"}, {"variable": "data"}),
                            (".npy", {}, {}),):
        for s in splits(3):
            path = _tmp("save_{}{}".format(s, ext))
            ht.save(ht.array(x, split=s), path, **kw)
            for ls in splits(3):
                same(ht.load(path, split=ls, **loadkw), x)
    m = np.arange(12.0).reshape(4, 3)
    for s in (None, 0, 1):
        path = _tmp("save_{}.csv".format(s))
        ht.save(ht.array(m, split=s), path)
        same(ht.load(path, split=0, dtype=ht.float64), m)


def test_save_exception():
    data = ht.arange(1)
    for p, k in ((_tmp("e.h5"), "data"), (_tmp("e.nc"), "data")):
        raises(TypeError, ht.save, 1, p, k)
        raises(TypeError, ht.save, data, 1, k)
        raises(TypeError, ht.save, data, p, 1)
    raises(ValueError, ht.save, data, _tmp("e.nc"), "data", mode="r")
    raises(ValueError, ht.save, 1, "data.dat")


def test_load_hdf5():
    ref = _iris_np()
    if ref is None:
        return
    a = ht.load_hdf5(H5, "data")
    assert a.gshape == (150, 4) and a.dtype == ht.float32 and a.split is None
    a = ht.load_hdf5(H5, "data", split=0)
    assert a.split == 0
    same(a, ref)
    a = ht.load_hdf5(H5, "data", split=-1)
    assert a.split == 1
    same(a, ref)
    a = ht.load_hdf5(H5, "data", dtype=ht.int8)
    assert a.dtype == ht.int8
    same(a, ref.astype(np.int8))


def test_load_hdf5_exception():
    raises(TypeError, ht.load_hdf5, 1, "data")
    raises(TypeError, ht.load_hdf5, "iris.h5", 1)
    raises(TypeError, ht.load_hdf5, "iris.h5", dataset="data", split=1.0)
    raises(IOError, ht.load_hdf5, "foo.h5", dataset="data")
    if os.path.exists(H5):
        raises(IOError, ht.load_hdf5, H5, dataset="foo")


def test_save_hdf5():
    x = np.arange(60, dtype=np.float64).reshape(12, 5)
    for s in splits(2):
        path = _tmp("h5_{}.h5".format(s))
        ht.save_hdf5(ht.array(x, split=s), path, "data")
        same(ht.load_hdf5(path, "data", dtype=ht.float64, split=0), x)
        # a second dataset in append mode keeps the first
        ht.save_hdf5(ht.array(x * 2, split=s), path, "twice", mode="a")
        same(ht.load_hdf5(path, "data", dtype=ht.float64), x)
        same(ht.load_hdf5(path, "twice", dtype=ht.float64, split=1), x * 2)


def test_save_hdf5_compressed():
    """``save_hdf5(..., compression="gzip", compression_opts, chunks, shuffle, fletcher32)`` (the
    reference forwards these to h5py, ``io.py:185-197``): chunked, filtered storage written in
    parallel (chunks crossing rank boundaries included) and read back through ``load_hdf5`` on
    every split, plus slab reads that decode only the touched chunks. Byte-level parity with
    h5py is unpinned (h5py is not importable here); the file layout follows the HDF5 spec."""
    from heat_amd.core import _h5lite

    rng = np.random.default_rng(3)
    x = np.round(rng.standard_normal((37, 6)), 2)
    cases = [dict(compression="gzip"), dict(compression="gzip", compression_opts=9, shuffle=True),
             dict(compression="gzip", compression_opts=1, chunks=(5, 4), fletcher32=True), dict(chunks=(7, 6)),
             dict(compression="gzip", chunks=(40, 2), shuffle=True)]
    for ci, kw in enumerate(cases):
        for s in splits(2):
            path = _tmp("h5z_{}_{}.h5".format(ci, s))
            ht.save_hdf5(ht.array(x, split=s), path, "data", **kw)
            for ls in (None, 0, 1):
                same(ht.load_hdf5(path, "data", dtype=ht.float64, split=ls), x)
            with _h5lite.open_file(path) as f:
                ds = f["data"]
                assert ds._layout["kind"] == "chunked"
                assert np.array_equal(ds[3:29, 1:5], x[3:29, 1:5])
                assert np.array_equal(ds[-1], x[-1])
                if "compression" in kw:
                    assert any(fid == 1 for fid, _ in ds._layout["filters"])
    # integers, a 1-D array and a second dataset appended to a compressed file
    v = np.arange(1000, dtype=np.int32) * 3
    path = _tmp("h5z_int.h5")
    ht.save_hdf5(ht.array(v, split=0), path, "v", compression="gzip", chunks=(64,))
    ht.save_hdf5(ht.array(x, split=0), path, "x", mode="a", compression="gzip", shuffle=True)
    same(ht.load_hdf5(path, "v", dtype=ht.int32, split=0), v)
    same(ht.load_hdf5(path, "x", dtype=ht.float64), x)
    # 200 chunks: a two-level chunk B-tree (64 entries per node)
    w = np.arange(2000, dtype=np.float32)
    ht.save_hdf5(ht.array(w, split=0), path, "many", mode="a", compression="gzip", chunks=(10,))
    same(ht.load_hdf5(path, "many", dtype=ht.float32, split=0), w)
    raises(NotImplementedError, ht.save_hdf5, ht.array(x), _tmp("h5z_bad.h5"), "d", compression="lzf")


def test_save_hdf5_exception():
    data = ht.arange(1)
    raises(TypeError, ht.save_hdf5, 1, _tmp("x.h5"), "data")
    raises(TypeError, ht.save_hdf5, data, 1, "data")
    raises(TypeError, ht.save_hdf5, data, _tmp("x.h5"), 1)


def test_load_netcdf():
    ref = _iris_np()
    if ref is None:
        return
    a = ht.load_netcdf(NC, "data")
    assert a.gshape == (150, 4) and a.dtype == ht.float32 and a.split is None
    for s in (0, -1):
        a = ht.load_netcdf(NC, "data", split=s)
        assert a.split == (s % 2)
        same(a, ref)
    a = ht.load_netcdf(NC, "data", dtype=ht.int8)
    assert a.dtype == ht.int8


def test_load_netcdf_exception():
    raises(TypeError, ht.load_netcdf, 1, "data")
    raises(TypeError, ht.load_netcdf, "iris.nc", variable=1)
    raises(TypeError, ht.load_netcdf, "iris.nc", variable="data", split=1.0)
    raises(IOError, ht.load_netcdf, "foo.nc", variable="data")
    if os.path.exists(NC):
        raises(IOError, ht.load_netcdf, NC, variable="foo")


def test_save_netcdf():
    x = np.arange(6 * 4, dtype=np.float32).reshape(6, 4)
    for s in splits(2):
        path = _tmp("nc_{}.nc".format(s))
        ht.save_netcdf(ht.array(x, split=s), path, "data")
        same(ht.load_netcdf(path, "data", split=0), x)
        # r+ overwrites a slice in place
        ht.save_netcdf(ht.array(x[:2] * 10, split=s), path, "data", mode="r+", file_slices=slice(0, 2))
        e = x.copy()
        e[:2] *= 10
        same(ht.load_netcdf(path, "data"), e)
        # a second variable appended
        ht.save_netcdf(ht.array(x + 1, split=s), path, "other", mode="a", dimension_names=["a", "b"])
        same(ht.load_netcdf(path, "other", split=1), x + 1)
    # unlimited (record) dimension grown by later writes
    path = _tmp("nc_unlim.nc")
    ht.save_netcdf(ht.array(x, split=0), path, "rec", is_unlimited=True)
    ht.save_netcdf(ht.array(x + 100, split=0), path, "rec", mode="r+", file_slices=slice(6, 12), is_unlimited=True)
    same(ht.load_netcdf(path, "rec"), np.concatenate([x, x + 100]))


def test_save_netcdf_exception():
    data = ht.arange(1)
    p = _tmp("ne.nc")
    raises(TypeError, ht.save_netcdf, 1, p, "data")
    raises(TypeError, ht.save_netcdf, data, 1, "data")
    raises(TypeError, ht.save_netcdf, data, p, 1)
    raises(TypeError, ht.save_netcdf, data, p, "data", dimension_names=1)
    raises(ValueError, ht.save_netcdf, data, p, "data", dimension_names=["a", "b"])
    raises(ValueError, ht.save_netcdf, data, p, "data", mode="x")


def test_remove_folder():
    """The reference's (commented-out) clean-up check ``test_io.py:624-629``: after saving into a
    scratch folder every rank can see the file, and once all ranks passed a barrier rank 0 removes
    the folder, which then no longer exists for anyone."""
    comm = ht.MPI_WORLD
    base = os.path.join(tempfile.gettempdir(), "heat_amd_rmdir_{}".format(os.environ.get("MASTER_PORT", os.getpid())))
    if comm.rank == 0:
        os.makedirs(base, exist_ok=True)
    comm.Barrier()
    path = os.path.join(base, "x.csv")
    ht.save_csv(ht.arange(12, dtype=ht.float32, split=0).reshape((4, 3)), path) if hasattr(ht, "save_csv") else \
        ht.save(ht.arange(12, dtype=ht.float32, split=0).reshape((4, 3)), path)
    comm.Barrier()
    assert os.path.exists(path)
    comm.Barrier()
    if comm.rank == 0:
        os.remove(path)
        os.rmdir(base)
    comm.Barrier()
    assert not os.path.exists(base)
