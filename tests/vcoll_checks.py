"""Variable-count collectives (Allgatherv / Alltoallv / Gatherv / Scatterv /
reduce-scatter, the v-variants RCCL does not have natively) with UNEVEN and EMPTY blocks, on the
default device: host tensors in the CPU suite (gloo), ``cuda:0`` tensors with 3 and 5 ranks
sharing the GPU box's card (``tests/test_gpu_dist.py``: every collective then goes through the
host-staging wrappers). Non-contiguous device views are passed where the API accepts them.
Every result is compared with a closed-form expectation."""
import numpy as np
import torch

import heat_amd as ht

MPI = ht.MPI


def _dev():
    return ht.get_device().torch_device


def _counts(p, pattern):
    """Uneven counts with empty blocks: rank r holds pattern[r % len(pattern)] rows."""
    c = [pattern[r % len(pattern)] for r in range(p)]
    return c, [sum(c[:r]) for r in range(p)]


def _block(r, rows, cols, dev, base=0.0):
    return (torch.arange(rows * cols, dtype=torch.float64, device=dev).reshape(rows, cols)
            + 1000.0 * r + base) if rows else torch.empty((0, cols), dtype=torch.float64, device=dev)


def check_allgatherv_uneven_empty():
    comm = ht.MPI_WORLD
    p, me, dev = comm.size, comm.rank, _dev()
    for pattern in ([3, 0, 1], [0, 2], [5, 0, 0, 1]):
        counts, displs = _counts(p, pattern)
        send = _block(me, counts[me], 4, dev)
        recv = torch.empty((sum(counts), 4), dtype=torch.float64, device=dev)
        comm.Allgatherv(send, (recv, counts, displs))
        ref = torch.cat([_block(r, counts[r], 4, dev) for r in range(p)])
        assert torch.equal(recv, ref), pattern
        # along axis 1 (columns), from a non-contiguous (transposed) view
        sendT = _block(me, counts[me], 3, dev).t()
        recvT = torch.empty((3, sum(counts)), dtype=torch.float64, device=dev)
        comm.Allgatherv(sendT, (recvT, counts, displs), recv_axis=1)
        assert torch.equal(recvT, torch.cat([_block(r, counts[r], 3, dev).t() for r in range(p)], 1))
        # allgather_tensor with unequal and empty row blocks
        got = comm.allgather_tensor(send, 0)
        assert torch.equal(got, ref)


def check_alltoallv_uneven_empty():
    comm = ht.MPI_WORLD
    p, me, dev = comm.size, comm.rank, _dev()
    # rank r sends (r + q) % 3 rows to rank q (0 rows where that is 0)
    sc = [(me + q) % 3 for q in range(p)]
    rc = [(q + me) % 3 for q in range(p)]
    sd = [sum(sc[:q]) for q in range(p)]
    rd = [sum(rc[:q]) for q in range(p)]
    s = torch.cat([torch.full((sc[q], 2), float(100 * me + q), device=dev, dtype=torch.float64)
                   for q in range(p)]) if sum(sc) else torch.empty((0, 2), dtype=torch.float64, device=dev)
    r = torch.full((sum(rc), 2), -1.0, dtype=torch.float64, device=dev)
    comm.Alltoallv((s, sc, sd), (r, rc, rd))
    ref = [torch.full((rc[q], 2), float(100 * q + me), device=dev, dtype=torch.float64) for q in range(p)]
    ref = torch.cat(ref) if sum(rc) else torch.empty((0, 2), dtype=torch.float64, device=dev)
    assert torch.equal(r, ref)
    # the split-axis exchange of a DNDarray whose ranks hold uneven / empty blocks
    n = 2 * p + 1
    a = np.arange(n * 3, dtype=np.float32).reshape(n, 3)
    x = ht.array(a, split=0)
    counts = [0 if q % 2 else 2 for q in range(p)]
    counts[-1] += n - sum(counts)
    x.redistribute_(lshape_map=x.create_lshape_map(), target_map=torch.tensor([[c, 3] for c in counts]))
    assert x.lshape[0] == counts[me]
    y = ht.resplit(x, 1)
    assert np.array_equal(y.numpy(), a) and y.split == 1


def check_gatherv_scatterv_uneven_empty():
    comm = ht.MPI_WORLD
    p, me, dev = comm.size, comm.rank, _dev()
    counts, displs = _counts(p, [2, 0, 3])
    root = p - 1
    send = _block(me, counts[me], 2, dev)
    out = torch.empty((sum(counts), 2), dtype=torch.float64, device=dev) if me == root else None
    comm.Gatherv(send, (out, counts, displs) if me == root else None, root=root)
    if me == root:
        assert torch.equal(out, torch.cat([_block(r, counts[r], 2, dev) for r in range(p)]))
    src = torch.cat([_block(r, counts[r], 2, dev, 0.5) for r in range(p)]) if me == 0 else None
    mine = torch.empty((counts[me], 2), dtype=torch.float64, device=dev)
    comm.Scatterv((src, counts, displs) if me == 0 else None, mine, root=0)
    assert torch.equal(mine, _block(me, counts[me], 2, dev, 0.5))


def check_reduce_scatter_uneven():
    """``reduce_scatter_tensor`` (the matmul contraction-split path) and the matmul itself with
    uneven blocks: rank r's block of the rank-sum, against the closed form."""
    comm = ht.MPI_WORLD
    p, me, dev = comm.size, comm.rank, _dev()
    inp = torch.arange(p * 6, dtype=torch.float64, device=dev).reshape(p * 2, 3) * (me + 1)
    out = torch.empty((2, 3), dtype=torch.float64, device=dev)
    comm.reduce_scatter_tensor(out, inp)
    tot = p * (p + 1) / 2
    ref = torch.arange(p * 6, dtype=torch.float64, device=dev).reshape(p * 2, 3)[2 * me: 2 * me + 2] * tot
    assert torch.equal(out, ref)
    rng = np.random.default_rng(5)
    for (m, k, n) in ((2 * p + 1, p + 2, 3), (3, 2 * p - 1, p + 1)):
        a = rng.standard_normal((m, k))
        b = rng.standard_normal((k, n))
        C = ht.array(a, split=1) @ ht.array(b, split=0)
        assert np.allclose(C.numpy(), a @ b, rtol=1e-10, atol=1e-12)


def check_exchange_empty_ranks_statistics():
    """Reductions and moments when some ranks hold nothing (more ranks than rows)."""
    comm = ht.MPI_WORLD
    p = comm.size
    n = max(1, p - 2)
    a = np.arange(n * 2, dtype=np.float32).reshape(n, 2) + 1
    x = ht.array(a, split=0)
    assert np.allclose(ht.sum(x, axis=0).numpy(), a.sum(0))
    assert np.allclose(ht.mean(x, axis=0).numpy(), a.mean(0))
    assert np.allclose(ht.var(x, axis=0).numpy(), a.var(0), atol=1e-6)
    assert np.allclose(ht.max(x).item(), a.max())
    assert int(ht.argmin(x).item()) == int(a.argmin())


def check_native_comm_byte_plans():
    """The byte counts / offsets the native RCCL communicator hands to ``ha_comm_alltoallv``
    (``parallel/native_comm.py``), run through a host model of that grouped send/receive, give
    exactly the gloo results of ``allgather_tensor`` and ``exchange_axis`` - uneven blocks, empty
    ranks, every axis (the native path itself needs several GPUs; its arithmetic does not)."""
    from heat_amd.core.communication import exchange_axis_bytes
    from heat_amd.ops import kernels as K
    from heat_amd.parallel import native_comm as nc

    comm = ht.MPI_WORLD
    p, me = comm.size, comm.rank

    def raw(t):
        t = t.contiguous()
        return t.view(torch.uint8).numpy().reshape(-1) if t.numel() else np.zeros(0, np.uint8)

    # all-gather of unequal row blocks (some ranks empty)
    counts = [(3 * r + 1) % 4 for r in range(p)]
    block = torch.arange(counts[me] * 5, dtype=torch.float64).reshape(counts[me], 5) + 1000 * me
    real = comm.allgather_tensor(block, 0, counts)
    plan = nc.allgatherv_plan(counts, me, 5 * 8)
    sims = nc.simulate_alltoallv(comm.allgather(raw(block)), comm.allgather(plan), [sum(counts) * 40] * p)
    assert np.array_equal(sims[me].view(np.float64).reshape(-1, 5), real.numpy())

    # personalised exchanges along every axis pair of a 3-D array with uneven counts
    shape = (7, 2 * p + 1, 5)
    g = np.arange(np.prod(shape), dtype=np.int32).reshape(shape)
    for split in range(3):
        for target in range(3):
            if split == target:
                continue
            scounts = comm.counts_displs_shape(shape, target)[0]
            rcounts = comm.counts_displs_shape(shape, split)[0]
            lo = sum(rcounts[:me])
            send = torch.from_numpy(np.ascontiguousarray(np.take(g, range(lo, lo + rcounts[me]), axis=split)))
            recv_shape = list(shape)
            recv_shape[target] = scounts[me]
            real = comm.exchange_axis(send, target, scounts, tuple(recv_shape), split, rcounts)
            in_b, out_b = exchange_axis_bytes(tuple(send.shape), target, scounts, tuple(recv_shape), split, rcounts,
                                              send.element_size())
            packed = K.pack_blocks(send, target, scounts)
            plans = comm.allgather(nc.alltoallv_plan(in_b, out_b))
            sends = comm.allgather(raw(packed))
            sizes = comm.allgather(int(sum(out_b)))
            sim = nc.simulate_alltoallv(sends, plans, sizes)[me]
            got = K.unpack_blocks(torch.from_numpy(sim.view(np.int32).copy()), tuple(recv_shape), split, rcounts)
            assert torch.equal(got, real), (split, target)
            t0 = sum(scounts[:me])
            assert np.array_equal(real.numpy(), np.take(g, range(t0, t0 + scounts[me]), axis=target))

    # a mismatched plan is caught (the real exchange would hang): rank 0 announces one byte more
    if p > 1:
        bad = [list(nc.alltoallv_plan([4] * p, [4] * p)) for _ in range(p)]
        bad[0][0] = bad[0][0].copy()
        bad[0][0][1] += 1
        try:
            nc.simulate_alltoallv([np.zeros(4 * p + 1, np.uint8)] * p, bad, [4 * p] * p)
        except ValueError:
            pass
        else:
            raise AssertionError("mismatched send/receive sizes not detected")
