"""
Rank bodies of the IPC all-reduce GPU test (``tests/test_gpu_ipc.py``): N processes share the
box's one MI355X, exchange hipIpc handles over gloo and all-reduce through the mapped buffers.
Every rank builds every rank's input from the same seed, so the exact expected sum (same
rank-order fp summation as the kernel) is known locally.
"""
from __future__ import annotations

import os

import numpy as np
import torch

import heat_amd as ht
from heat_amd.parallel.ipc import IpcAllreduce


def _inputs(it: int, n: int, p: int, dtype):
    g = torch.Generator().manual_seed(7919 * it + n)
    full = torch.randn(p, n, generator=g, dtype=torch.float64)
    if dtype == torch.int64:
        full = (full * 1000).round()
    full = full.to(dtype)
    ref = full[0].clone()
    for q in range(1, p):
        ref += full[q]
    return full, ref


def check_ipc_allreduce():
    comm = ht.MPI_WORLD
    p, r = comm.size, comm.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    ar = IpcAllreduce(comm, capacity_bytes=1 << 20, blocks=16, timeout_spins=2_000_000)
    cases = ((torch.float32, 1), (torch.float32, 1000), (torch.float64, 66560), (torch.int64, 777),
             (torch.float32, 262144), (torch.float64, 3))
    for it in range(20):
        for dtype, n in cases:
            full, ref = _inputs(it, n, p, dtype)
            t = full[r].clone().to(dev)
            ar.allreduce_(t)
            got = t.cpu()
            assert torch.equal(got, ref), (it, dtype, n, (got.double() - ref.double()).abs().max().item())
    # back-to-back calls without host synchronisation (slot reuse + epoch ordering)
    ts = []
    for it in range(50):
        full, ref = _inputs(100 + it, 4096, p, torch.float32)
        t = full[r].clone().to(dev)
        ar.allreduce_(t)
        ts.append((t, ref))
    for t, ref in ts:
        assert torch.equal(t.cpu(), ref)
    assert ar.error() == 0, "an IPC barrier timed out"
    ar.close()


def check_ipc_through_communication():
    """``MPICommunication.Allreduce`` routes small device SUMs through the IPC kernel when
    HEAT_IPC_ALLREDUCE=1 (set by the test); results equal the rank-order sum."""
    assert os.environ.get("HEAT_IPC_ALLREDUCE") == "1"
    comm = ht.MPI_WORLD
    p, r = comm.size, comm.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    for it in range(5):
        full, ref = _inputs(500 + it, 1024 * 65 + 1024, p, torch.float64)
        t = full[r].clone().to(dev)
        comm.Allreduce(ht.MPI.IN_PLACE, t, ht.MPI.SUM)
        assert torch.equal(t.cpu(), ref)
    assert getattr(comm, "_ipc", None) is not None, "the IPC path was not taken"
    # a distributed reduction of the op engine (sum over the split axis) on the device
    x = ht.arange(4000, dtype=ht.float64, split=0, device="gpu")
    assert x.larray.is_cuda
    assert ht.sum(x).item() == 4000 * 3999 / 2
    assert comm._ipc.error() == 0


def check_ipc_timeout_is_loud():
    """A rank that never joins: the waiting rank's output is NaN-poisoned and the NEXT call (or
    check()) raises IpcTimeoutError - never a silently wrong sum."""
    import time

    from heat_amd.parallel.ipc import IpcTimeoutError

    comm = ht.MPI_WORLD
    r = comm.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    ar = IpcAllreduce(comm, capacity_bytes=1 << 16, blocks=4, timeout_spins=2_000_000)
    t = torch.ones(1000, device=dev)
    ar.allreduce_(t)                                   # a good call first
    ar.check()
    assert torch.equal(t.cpu(), torch.full((1000,), float(comm.size)))
    comm.Barrier()
    if r == 0:
        ar.spins = 2000                                # a short bound for the call nobody joins
        t = torch.ones(1000, device=dev)
        ar.allreduce_(t)                               # the peers sit out this call
        torch.cuda.synchronize()
        assert torch.isnan(t).all(), "a timed-out call must not return a sum"
        try:
            ar.check()
            raise AssertionError("check() must raise after a timeout")
        except IpcTimeoutError:
            pass
        try:
            ar.allreduce_(torch.ones(10, device=dev))
            raise AssertionError("a poisoned communicator must refuse further calls")
        except IpcTimeoutError:
            pass
    else:
        time.sleep(0.5)
    comm.Barrier()


def check_ipc_allgather_and_two_shot():
    """Direct W-peer all-gather (uneven and empty blocks, float32 / int64 / bf16 rows) and the
    two-shot all-reduce above the threshold, against host-built expectations; then the same
    through ``MPICommunication.allgather_tensor`` with HEAT_IPC_ALLREDUCE=1."""
    comm = ht.MPI_WORLD
    p, r = comm.size, comm.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    ar = IpcAllreduce(comm, capacity_bytes=4 << 20, blocks=16, timeout_spins=2_000_000)
    for it in range(10):
        for dtype, width in ((torch.float32, 3), (torch.int64, 1), (torch.bfloat16, 4)):
            g = torch.Generator().manual_seed(31 * it + width)
            counts = [int(c) for c in torch.randint(0, 700, (p,), generator=g)]
            if it == 0:
                counts[0] = 0
            blocks = [(torch.randn(c, width, generator=g) * 100).to(dtype) for c in counts]
            row = width * torch.tensor([], dtype=dtype).element_size()
            out = ar.allgather(blocks[r].to(dev).contiguous(), [c * row for c in counts])
            assert out is not None
            got = out.view(dtype).reshape(-1, width).cpu()
            assert torch.equal(got, torch.cat(blocks)), (it, dtype)
    # two-shot all-reduce (payload > HEAT_IPC_TWOSHOT_BYTES), including n not divisible by p
    for n in (300_001, 1 << 19):
        full, ref = _inputs(900 + n, n, p, torch.float32)
        t = full[r].clone().to(dev)
        ar.allreduce_(t)
        assert torch.equal(t.cpu(), ref)
    ar.check()
    ar.close()
    os.environ["HEAT_IPC_ALLREDUCE"] = "1"
    x = torch.arange(r * 10, r * 10 + 10 + r, dtype=torch.float32, device=dev).reshape(-1, 1).repeat(1, 4)
    allx = comm.allgather_tensor(x, 0)
    exp = torch.cat([torch.arange(q * 10, q * 10 + 10 + q, dtype=torch.float32).reshape(-1, 1).repeat(1, 4)
                     for q in range(p)])
    assert torch.equal(allx.cpu(), exp)
    assert getattr(comm, "_ipc", None) is not None, "the IPC all-gather was not taken"
    y = ht.random.randn(1000, 8, split=0, device="gpu")
    yn = y.numpy()  # gathers through the IPC path
    assert yn.shape == (1000, 8)
    comm._ipc.check()


def bench_ipc():
    """Latency / bandwidth of the IPC collectives vs payload (rank 0 prints JSON lines). With the
    ranks sharing one GPU the 'links' are local HBM: this measures the protocol (launch, barriers,
    copies), not xGMI."""
    import json
    import time

    comm = ht.MPI_WORLD
    p, r = comm.size, comm.rank
    dev = torch.device("cuda", torch.cuda.current_device())
    ar = IpcAllreduce(comm, capacity_bytes=64 << 20, blocks=64, timeout_spins=50_000_000)
    for nbytes in (4 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
        t = torch.ones(nbytes // 4, device=dev)
        res = {"world": p, "bytes": nbytes}
        for name, ts in (("one_shot", 1 << 62), ("two_shot", 0)):
            ar.two_shot_bytes = ts
            for _ in range(3):
                ar.allreduce_(t)
            torch.cuda.synchronize()
            comm.Barrier()
            reps = 20
            t0 = time.perf_counter()
            for _ in range(reps):
                ar.allreduce_(t)
            torch.cuda.synchronize()
            res[name + "_us"] = round((time.perf_counter() - t0) / reps * 1e6, 1)
        blk = torch.ones(nbytes // 4 // p, device=dev)
        for _ in range(3):
            ar.allgather(blk, [blk.numel() * 4] * p)
        torch.cuda.synchronize()
        comm.Barrier()
        t0 = time.perf_counter()
        for _ in range(20):
            ar.allgather(blk, [blk.numel() * 4] * p)
        torch.cuda.synchronize()
        res["allgather_us"] = round((time.perf_counter() - t0) / 20 * 1e6, 1)
        if r == 0:
            print(json.dumps(res), flush=True)
    ar.check()
    ar.close()


def check_ipc_halo():
    """``DNDarray.get_halo`` takes the xGMI peer path under HEAT_IPC_ALLREDUCE=1: every rank's
    boundary slices in one direct all-gather kernel; neighbours' slices match the data (split 0
    and split 1, halo 1 and 3), and ``diff`` along the split axis agrees with numpy."""
    assert os.environ.get("HEAT_IPC_ALLREDUCE") == "1"
    comm = ht.MPI_WORLD
    r, p = comm.rank, comm.size
    a = np.arange(24 * 10, dtype=np.float32).reshape(24, 10)
    for split in (0, 1):
        x = ht.array(a, split=split, device="gpu")
        assert x.larray.is_cuda
        counts, displs = x.counts_displs()
        for h in (1, 3):
            x.get_halo(h)
            if r > 0:
                lo = displs[r] - h
                ref = a[lo: displs[r]] if split == 0 else a[:, lo: displs[r]]
                assert np.array_equal(x.halo_prev.cpu().numpy(), ref), (split, h)
            else:
                assert x.halo_prev is None
            if r < p - 1:
                hi = displs[r] + counts[r]
                ref = a[hi: hi + h] if split == 0 else a[:, hi: hi + h]
                assert np.array_equal(x.halo_next.cpu().numpy(), ref), (split, h)
            else:
                assert x.halo_next is None
        assert np.allclose(ht.diff(x, axis=split).numpy(), np.diff(a, axis=split))
    assert getattr(comm, "_ipc", None) is not None, "the IPC path was not taken"
    assert comm._ipc.error() == 0


def check_ipc_iterative_paths():
    """The latency-bound iterative paths ride the IPC one-shot when HEAT_IPC_ALLREDUCE=1: the
    distributed Householder QR (one fp64 column-sum all-reduce per column) and Lanczos (two
    all-reduces per step) take ``allreduce:ipc`` (PATH_COUNTS) and stay correct."""
    from heat_amd.core.communication import PATH_COUNTS

    assert os.environ.get("HEAT_IPC_ALLREDUCE") == "1"
    comm = ht.MPI_WORLD
    rng = np.random.default_rng(11)
    a_np = rng.standard_normal((300, 40))
    before = PATH_COUNTS["allreduce:ipc"]
    q, r = ht.linalg.qr(ht.array(a_np, split=0, device="gpu"), mode="complete")
    qq, rr = q.numpy(), r.numpy()
    assert np.allclose(qq @ rr, a_np, atol=1e-8)
    assert np.allclose(qq.T @ qq, np.eye(300), atol=1e-8)
    hh = PATH_COUNTS["allreduce:ipc"] - before
    assert hh >= 40, hh                     # at least one per column
    spd = a_np.T @ a_np + np.eye(40)
    before = PATH_COUNTS["allreduce:ipc"]
    V, T = ht.lanczos(ht.array(spd, split=0, device="gpu"), 12,
                      v0=ht.array(np.ones(40) / np.sqrt(40), split=0, device="gpu"))
    vv = V.numpy()
    assert np.allclose(vv.T @ vv, np.eye(12), atol=1e-8)
    assert PATH_COUNTS["allreduce:ipc"] - before >= 2 * 11
    assert comm._ipc.error() == 0
    if comm.rank == 0:
        print("PATH_COUNTS", dict(PATH_COUNTS), flush=True)
