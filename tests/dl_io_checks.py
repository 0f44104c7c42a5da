"""Adversarial checks of the deep-learning and IO layer, run at 2-8 gloo ranks (and at one rank in
``test_core_local.py``-style single runs): the silent-corruption paths found in review.

* ``DataParallel`` with a parameter that never gets a gradient (its bucket must still be
  averaged, every rank must hold the same parameters, equal to a single-process run on the
  union of the rank batches); blocking and deferred updates, one bucket and many buckets.
* ``PartialH5Dataset`` whose loader is slower than the consumer: every row of the rank's share
  is seen exactly once per epoch, several epochs in a row; ``validate_set``; ``len``.
* netCDF without the netCDF4 package: int64 ``2**40`` and uint8 ``200`` survive a round trip
  bit-exactly, and a NumPy read of the raw file bytes shows the same values.
"""
import os
import tempfile
import time

import numpy as np
import torch

import heat_amd as ht


class _NetWithUnused(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(4, 8)
        self.unused = torch.nn.Linear(8, 8)     # never called in forward
        self.b = torch.nn.Linear(8, 1)

    def forward(self, x):
        return self.b(torch.relu(self.a(x)))


def _dev():
    """cuda when the ranks run with device buffers (tests/test_gpu_dist.py), else cpu."""
    on = os.environ.get("HEAT_AMD_DEFAULT_DEVICE") == "gpu" and torch.cuda.is_available()
    return torch.device("cuda", 0) if on else torch.device("cpu")


def _dp_run(blocking: bool, bucket_mb: float, steps: int = 3, momentum: float = 0.0):
    comm = ht.MPI_WORLD
    dev = _dev()
    torch.manual_seed(0)
    net = _NetWithUnused().to(dev)
    opt = ht.optim.DataParallelOptimizer(torch.optim.SGD(net.parameters(), lr=0.1, momentum=momentum),
                                         blocking=blocking)
    dp = ht.nn.DataParallel(net, comm, opt, blocking_parameter_updates=blocking, bucket_cap_mb=bucket_mb)
    ref = _NetWithUnused().to(dev)
    ref.load_state_dict(net.state_dict())
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=momentum)
    g = torch.Generator().manual_seed(7)
    per = 5
    for _ in range(steps):
        Xg = torch.randn(per * comm.size, 4, generator=g).to(dev)
        yg = torch.randn(per * comm.size, 1, generator=g).to(dev)
        sl = slice(comm.rank * per, (comm.rank + 1) * per)     # per-rank data
        opt.zero_grad()
        torch.nn.functional.mse_loss(dp(Xg[sl]), yg[sl]).backward()
        opt.step()
        ref_opt.zero_grad()
        torch.nn.functional.mse_loss(ref(Xg), yg).backward()
        ref_opt.step()
    dp.eval()  # finalises a deferred (non-blocking) update
    flat = torch.cat([p.detach().reshape(-1) for p in net.parameters()]).cpu()
    allflat = comm.allgather(flat.numpy())
    for r, other in enumerate(allflat):
        assert np.array_equal(other, allflat[0]), "rank {} diverged from rank 0".format(r)
    for (n, p), q in zip(net.named_parameters(), ref.parameters()):
        assert torch.allclose(p, q, atol=1e-5), (n, p, q)
    assert net.unused.weight.grad is None  # never touched, like the reference (no hook fires)


def check_dp_unused_parameter_blocking():
    _dp_run(blocking=True, bucket_mb=25.0)          # one bucket holding the unused layer
    _dp_run(blocking=True, bucket_mb=0.0001)        # one bucket per parameter
    _dp_run(blocking=True, bucket_mb=25.0, momentum=0.9)


def check_dp_unused_parameter_nonblocking():
    _dp_run(blocking=False, bucket_mb=25.0)
    _dp_run(blocking=False, bucket_mb=0.0002)


def _h5_file(comm, n, ncols=3):
    d = comm.bcast(tempfile.mkdtemp() if comm.rank == 0 else None, root=0)
    data = np.arange(n * ncols, dtype=np.float32).reshape(n, ncols)
    labels = np.arange(n, dtype=np.float32)
    path = os.path.join(d, "p.h5")
    ht.save_hdf5(ht.array(data, split=0), path, "data")
    ht.save_hdf5(ht.array(labels, split=0), path, "labels", mode="a")
    return path


def check_partial_h5_slow_loader_sees_every_row():
    comm = ht.MPI_WORLD
    n = 103 * comm.size + 3           # tail rows beyond size * (n // size) belong to nobody
    path = _h5_file(comm, n)
    ds = ht.utils.data.PartialH5Dataset(path, comm=comm, dataset_names=["data", "labels"], use_gpu=False,
                                        initial_load=20, load_length=16)
    assert len(ds) == n
    share = n // comm.size
    orig = ds._read

    def slow_read(lo, hi):
        time.sleep(0.05)
        return orig(lo, hi)

    ds._read = slow_read
    loader = ht.utils.data.DataLoader(ds, batch_size=4)
    assert len(loader) == share // 4
    lo = comm.rank * share
    for epoch in range(3):
        seen = []
        for x, y in loader:
            assert x.shape[0] == 4
            assert torch.equal(x[:, 0] / 3, y)
            seen.append(y)
        got = torch.cat(seen).long().tolist()
        assert len(got) == len(set(got)) == (share // 4) * 4, (epoch, len(got), share)
        assert set(got) <= set(range(lo, lo + share))
    # batch size 1: every row of the share
    loader = ht.utils.data.DataLoader(ds, batch_size=1)
    seen = torch.cat([y for _, y in loader]).long().tolist()
    assert sorted(seen) == list(range(lo, lo + share))


def check_partial_h5_break_then_full_epoch():
    """A consumer that breaks out of an epoch (after moving past window 0, and within window 0)
    must not leave the loader blocked on its bounded queue: the next epoch starts, and sees every
    row of the share exactly once (4+ windows)."""
    comm = ht.MPI_WORLD
    n = 97 * comm.size
    path = _h5_file(comm, n)
    ds = ht.utils.data.PartialH5Dataset(path, comm=comm, dataset_names=["data", "labels"], use_gpu=False,
                                        initial_load=10, load_length=8)
    share = n // comm.size
    assert len(ds.windows) >= 4
    lo = comm.rank * share
    for stop_after in (5, 1, 0, 23):    # batches consumed before the break (5 and 23: past window 0)
        loader = ht.utils.data.DataLoader(ds, batch_size=2)
        t0 = time.time()
        for i, _ in enumerate(loader):
            if i + 1 >= stop_after:
                break
        time.sleep(0.2)                 # the abandoned loader fills its queue and blocks
        loader = ht.utils.data.DataLoader(ds, batch_size=1)
        seen = torch.cat([y for _, y in loader]).long().tolist()
        assert sorted(seen) == list(range(lo, lo + share)), stop_after
        assert time.time() - t0 < 60
    assert ds.load_thread is None or not ds.load_thread.is_alive() or ds._epoch_done


def check_partial_h5_drop_last_big_batches():
    """drop_last with batch_size > load_length: the leftover rows of an epoch sit in windows the
    consumer never fetched, so the loader is still blocked on its bounded queue when the epoch
    ends. The next epoch must cancel it (not join it) and still see every full batch."""
    comm = ht.MPI_WORLD
    n = 67 * comm.size
    path = _h5_file(comm, n)
    ds = ht.utils.data.PartialH5Dataset(path, comm=comm, dataset_names=["data", "labels"], use_gpu=False,
                                        initial_load=6, load_length=3)
    share = n // comm.size
    lo = comm.rank * share
    t0 = time.time()
    for epoch in range(3):
        loader = ht.utils.data.DataLoader(ds, batch_size=16, drop_last=True)
        got = torch.cat([y for _, y in loader]).long().tolist()
        assert len(got) == len(set(got)) == (share // 16) * 16, (epoch, len(got))
        assert set(got) <= set(range(lo, lo + share))
        time.sleep(0.1)                 # the loader fills its queue with the unfetched windows
    assert time.time() - t0 < 60
    assert ds.loads_remaining >= 0


def check_partial_h5_validate_set():
    comm = ht.MPI_WORLD
    n = 9 * comm.size + 1
    path = _h5_file(comm, n)
    ds = ht.utils.data.PartialH5Dataset(path, comm=comm, dataset_names=["data", "labels"], use_gpu=False,
                                        validate_set=True, initial_load=4, load_length=2)
    assert not ds.partial_dataset and len(ds) == n
    loader = ht.utils.data.DataLoader(ds, batch_size=1)
    seen = torch.cat([y for _, y in loader]).long().tolist()
    assert sorted(seen) == list(range(n))   # the whole file on every rank
    big = ht.utils.data.PartialH5Dataset(path, comm=comm, dataset_names="labels", use_gpu=False,
                                         initial_load=10 ** 6)
    assert not big.partial_dataset and big.length == n


def check_netcdf_lossless_int64_uint8_bool():
    from heat_amd.core import _ncclassic as ncc

    comm = ht.MPI_WORLD
    d = comm.bcast(tempfile.mkdtemp() if comm.rank == 0 else None, root=0)
    cases = {
        "i64": np.array([1, 2 ** 40, -3, -(2 ** 62), 7, 2 ** 53 + 1] * comm.size, dtype=np.int64),
        "u8": np.array([200, 0, 255, 1, 128, 3] * comm.size, dtype=np.uint8),
        "b": np.array([True, False, True, True, False, False] * comm.size),
        "u4": np.array([2 ** 32 - 1, 5, 0, 1, 2, 3] * comm.size, dtype=np.uint32),
    }
    for name, arr in cases.items():
        p = os.path.join(d, name + ".nc")
        for split in (None, 0):
            ht.save_netcdf(ht.array(arr, split=split), p, "v")
            ht_dtype = ht.int64 if arr.dtype == np.uint32 else ht.types.canonical_heat_type(arr.dtype)
            back = ht.load_netcdf(p, "v", dtype=ht_dtype).numpy()
            assert np.array_equal(back, arr), (name, back, arr)
        if comm.rank == 0:
            with open(p, "rb") as f:
                assert f.read(4) == b"CDF\x05"          # 64-bit data format
            shape, dt, begin, _ = ncc.layout(ncc.parse(p), "v")
            raw = np.fromfile(p, dtype=dt, count=arr.size, offset=begin)  # independent raw read
            assert np.array_equal(raw.astype(arr.dtype), arr), (name, raw)
        comm.Barrier()
    # 2-D int64 appended to an existing CDF-2 float file: the file is promoted, old data kept
    p = os.path.join(d, "mix.nc")
    f = np.arange(6 * comm.size * 2, dtype=np.float32).reshape(6 * comm.size, 2)
    ht.save_netcdf(ht.array(f, split=0), p, "f")
    if comm.rank == 0:
        with open(p, "rb") as fh:
            assert fh.read(4) == b"CDF\x02"
    comm.Barrier()
    big = (np.arange(f.size, dtype=np.int64) * (2 ** 35)).reshape(f.shape)
    ht.save_netcdf(ht.array(big, split=1), p, "g", mode="a", dimension_names=["f_dim_0", "f_dim_1"])
    assert np.array_equal(ht.load_netcdf(p, "f", split=0).numpy(), f)
    assert np.array_equal(ht.load_netcdf(p, "g", dtype=ht.int64, split=0).numpy(), big)
    # complex data has no netCDF type: an error on every rank, no silent cast
    try:
        ht.save_netcdf(ht.array(np.ones(4, dtype=np.complex64)), os.path.join(d, "c.nc"), "c")
    except TypeError:
        pass
    else:
        raise AssertionError("complex netCDF write did not raise")
