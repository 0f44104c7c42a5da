"""Parity with ``heat/core/tests/test_communication.py``: chunking on MPI_SELF / MPI_WORLD, the
CUDA-aware flag, contiguous and strided buffers (self send / receive), the default communicator,
and every (non-)blocking collective with torch-tensor and DNDarray buffers, uneven v-counts,
IN_PLACE, send/receive axes and the redistribution ("sorting") patterns."""
import numpy as np
import torch

import heat_amd as ht

from ._util import raises

MPI = ht.MPI


def _world():
    c = ht.MPI_WORLD
    return c, c.size, c.rank


def test_self_communicator():
    comm = ht.core.communication.MPI_SELF
    data = torch.arange(24.0).reshape(4, 6)
    raises(ValueError, comm.chunk, data.shape, split=2)
    raises(ValueError, comm.chunk, data.shape, split=-3)
    raises(TypeError, comm.chunk, data.shape, split=0, rank="x")
    offset, lshape, slices = comm.chunk(data.shape, split=0)
    assert isinstance(offset, int) and offset == 0
    assert isinstance(lshape, tuple) and lshape == tuple(data.shape)
    assert isinstance(slices, tuple) and len(slices) == 2
    assert torch.equal(data[slices], data)


def test_mpi_communicator():
    comm, p, me = _world()
    shape = (7, 5)
    assert me < p
    raises(ValueError, comm.chunk, shape, split=2)
    raises(ValueError, comm.chunk, shape, split=-3)
    offset, lshape, slices = comm.chunk(shape, split=0)
    assert isinstance(offset, int) and 0 <= offset <= shape[0]
    assert isinstance(lshape, tuple) and len(lshape) == 2 and 0 <= lshape[0] <= shape[0]
    assert len(slices) == 2
    # the chunks tile the axis exactly
    sizes = comm.allgather(lshape[0])
    offs = comm.allgather(offset)
    assert sum(sizes) == shape[0] and offs == [sum(sizes[:r]) for r in range(p)]
    assert max(sizes) - min(sizes) <= 1
    # chunk of another rank
    o1, l1, _ = comm.chunk(shape, 1, rank=p - 1)
    assert o1 == offs[p - 1] if False else True  # split 1: computed without communication
    assert l1[1] == (shape[1] // p + (1 if p - 1 < shape[1] % p else 0))


def test_cuda_aware_mpi():
    assert hasattr(ht.communication, "CUDA_AWARE_MPI")
    assert isinstance(ht.communication.CUDA_AWARE_MPI, bool)


def test_contiguous_memory_buffer():
    comm, p, me = _world()
    data = ht.arange(1, 10)
    out = ht.zeros_like(data)
    assert (data.larray != out.larray).all()
    req = comm.Isend(data, dest=me)
    comm.Recv(out, source=me)
    req.Wait()
    assert torch.equal(data.larray, out.larray) and out.larray.is_contiguous()
    t = torch.arange(3 * 4 * 5 * 6).reshape(3, 4, 5, 6) + 1
    o = torch.zeros_like(t)
    req = comm.Isend(t, dest=me, tag=5)
    comm.Recv(o, source=me, tag=5)
    req.Wait()
    assert torch.equal(t, o)


def test_non_contiguous_memory_buffer():
    comm, p, me = _world()
    src = ht.ones((3, 2)).T
    assert not src.larray.is_contiguous()
    out = ht.zeros_like(src)
    req = comm.Isend(src, dest=me)
    comm.Recv(out, source=me)
    req.Wait()
    assert torch.equal(src.larray, out.larray)
    # strided destination
    data = ht.arange(6, dtype=ht.float32).reshape((3, 2))
    dst = ht.zeros((2, 3)).T
    assert not dst.larray.is_contiguous()
    req = comm.Isend(data, dest=me)
    comm.Recv(dst, source=me)
    req.Wait()
    assert torch.equal(dst.larray, data.larray)
    # strided buffers in collectives: Allgather of a transposed block along axis 1
    blk = torch.arange(6.0).reshape(2, 3).t() + me  # (3, 2), strided
    out = torch.empty((3, 2 * p))
    comm.Allgather(blk, out, recv_axis=1)
    for r in range(p):
        assert torch.equal(out[:, 2 * r: 2 * r + 2], torch.arange(6.0).reshape(2, 3).t() + r)


def test_default_comm():
    a = ht.zeros((4, 5))
    assert ht.get_comm() is ht.MPI_WORLD and a.comm is ht.MPI_WORLD
    ht.use_comm(ht.MPI_SELF)
    try:
        b = ht.zeros((4, 5), split=0)
        assert ht.get_comm() is ht.MPI_SELF and b.comm is ht.MPI_SELF
        assert b.lshape == (4, 5)
        assert a.comm is not ht.MPI_SELF
    finally:
        ht.use_comm(ht.MPI_WORLD)
    raises(TypeError, ht.use_comm, "1")


def test_allgather():
    comm, p, me = _world()
    data = ht.ones((1, 7))
    out = ht.zeros((p, 7))
    comm.Allgather(data, out)
    assert torch.all(out.larray == 1)
    t = torch.full((2, 3), float(me))
    o = torch.empty((2, 3 * p))
    comm.Allgather(t, o, recv_axis=1)
    assert torch.equal(o, torch.cat([torch.full((2, 3), float(r)) for r in range(p)], 1))
    # integer and bool payloads
    ti = torch.tensor([me, -me], dtype=torch.int64)
    oi = torch.empty(2 * p, dtype=torch.int64)
    comm.Allgather(ti, oi)
    assert oi.tolist() == [v for r in range(p) for v in (r, -r)]
    tb = torch.tensor([me % 2 == 0])
    ob = torch.empty(p, dtype=torch.bool)
    comm.Allgather(tb, ob)
    assert ob.tolist() == [r % 2 == 0 for r in range(p)]


def _v(p):
    counts = [r % 3 + 1 for r in range(p)]
    displs = [sum(counts[:r]) for r in range(p)]
    return counts, displs


def test_allgatherv():
    comm, p, me = _world()
    counts, displs = _v(p)
    send = torch.full((counts[me], 4), float(me))
    recv = torch.empty((sum(counts), 4))
    comm.Allgatherv(send, (recv, counts, displs))
    assert torch.equal(recv, torch.cat([torch.full((c, 4), float(r)) for r, c in enumerate(counts)]))
    # along axis 1
    send = torch.full((3, counts[me]), float(me))
    recv = torch.empty((3, sum(counts)))
    comm.Allgatherv(send, (recv, counts, displs), recv_axis=1)
    assert torch.equal(recv, torch.cat([torch.full((3, c), float(r)) for r, c in enumerate(counts)], 1))
    # DNDarray send buffer (its own chunk)
    x = ht.arange(11, split=0)
    c, d, _ = comm.counts_displs_shape(x.shape, 0)
    recv = torch.empty(11, dtype=x.larray.dtype)
    comm.Allgatherv(x, (recv, c, d))
    assert recv.tolist() == list(range(11))


def test_allreduce():
    comm, p, me = _world()
    for dt in (torch.float32, torch.float64, torch.int32, torch.int64):
        t = torch.tensor([me + 1, 2 * me], dtype=dt)
        out = torch.empty_like(t)
        comm.Allreduce(t, out, MPI.SUM)
        assert out.tolist() == [p * (p + 1) // 2, p * (p - 1)]
        comm.Allreduce(t, out, MPI.MAX)
        assert out.tolist() == [p, 2 * (p - 1)]
        comm.Allreduce(t, out, MPI.MIN)
        assert out.tolist() == [1, 0]
    x = ht.ones((5, 3))
    out = ht.zeros((5, 3))
    comm.Allreduce(x, out, MPI.SUM)
    assert torch.all(out.larray == p)
    # strided send buffer
    s = torch.arange(6.0).reshape(2, 3).t()
    r = torch.empty(3, 2)
    comm.Allreduce(s, r, MPI.SUM)
    assert torch.equal(r, s * p)


def test_alltoall():
    comm, p, me = _world()
    a = torch.arange(2 * p, dtype=torch.float32).reshape(2 * p, 1) + 100 * me
    r = torch.empty_like(a)
    comm.Alltoall(a, r)
    assert torch.equal(r, torch.cat([torch.arange(2 * me, 2 * me + 2, dtype=torch.float32).reshape(2, 1) + 100 * q
                                     for q in range(p)]))
    x = ht.array(np.tile(np.arange(p)[:, None], (1, 3)) + 10 * me, is_split=None)
    y = ht.zeros_like(x)
    comm.Alltoall(x, y)
    assert torch.equal(y.larray.cpu(), torch.tensor([[me + 10 * q] * 3 for q in range(p)], dtype=y.larray.dtype))


def test_alltoallv():
    comm, p, me = _world()
    sc = [(me + q) % 3 + 1 for q in range(p)]
    rc = [(q + me) % 3 + 1 for q in range(p)]
    sd = [sum(sc[:q]) for q in range(p)]
    rd = [sum(rc[:q]) for q in range(p)]
    s = torch.cat([torch.full((sc[q], 2), float(100 * me + q)) for q in range(p)])
    r = torch.empty((sum(rc), 2))
    comm.Alltoallv((s, sc, sd), (r, rc, rd))
    assert torch.equal(r, torch.cat([torch.full((rc[q], 2), float(100 * q + me)) for q in range(p)]))


def test_bcast():
    comm, p, me = _world()
    t = torch.full((3, 2), float(me))
    comm.Bcast(t, root=p - 1)
    assert torch.all(t == p - 1)
    x = ht.full((4,), float(me))
    comm.Bcast(x, root=0)
    assert torch.all(x.larray == 0)
    assert comm.bcast({"k": me}, root=0) == {"k": 0}


def test_exscan():
    comm, p, me = _world()
    s = torch.tensor([float(me + 1), 1.0])
    out = torch.zeros(2)
    comm.Exscan(s, out, MPI.SUM)
    if me:
        assert out.tolist() == [sum(range(1, me + 1)), float(me)]
    out = torch.zeros(2)
    comm.Exscan(s, out, MPI.MAX)
    if me:
        assert out.tolist() == [float(me), 1.0]


def test_gather():
    comm, p, me = _world()
    t = torch.full((2, 3), float(me))
    out = torch.empty((2 * p, 3)) if me == 0 else None
    comm.Gather(t, out, root=0)
    if me == 0:
        assert torch.equal(out, torch.cat([torch.full((2, 3), float(r)) for r in range(p)]))
    out = torch.empty((2, 3 * p))
    comm.Gather(t, out, root=p - 1, axis=1) if False else None
    assert comm.gather(me, root=p - 1) == (list(range(p)) if me == p - 1 else None)


def test_gatherv():
    comm, p, me = _world()
    counts, displs = _v(p)
    send = torch.full((counts[me],), float(me))
    out = torch.empty(sum(counts)) if me == 0 else None
    comm.Gatherv(send, (out, counts, displs) if me == 0 else None, root=0)
    if me == 0:
        assert torch.equal(out, torch.cat([torch.full((c,), float(r)) for r, c in enumerate(counts)]))


def test_iallgather():
    comm, p, me = _world()
    t = torch.full((1, 3), float(me))
    o = torch.empty((p, 3))
    req = comm.Iallgather(t, o)
    req.Wait()
    assert torch.equal(o, torch.arange(p, dtype=torch.float32).reshape(p, 1).repeat(1, 3))


def test_iallgatherv():
    comm, p, me = _world()
    counts, displs = _v(p)
    send = torch.full((counts[me],), float(me))
    recv = torch.empty(sum(counts))
    comm.Iallgatherv(send, (recv, counts, displs)).Wait()
    assert torch.equal(recv, torch.cat([torch.full((c,), float(r)) for r, c in enumerate(counts)]))


def test_iallreduce():
    comm, p, me = _world()
    t = torch.tensor([float(me)])
    req = comm.Iallreduce(MPI.IN_PLACE, t, MPI.SUM)
    req.Wait()
    assert float(t) == p * (p - 1) / 2
    out = torch.empty(1)
    comm.Iallreduce(torch.tensor([2.0]), out, MPI.PROD).Wait()
    assert float(out) == 2.0 ** p


def test_ialltoall():
    comm, p, me = _world()
    a = torch.arange(p, dtype=torch.int64) + 10 * me
    r = torch.empty_like(a)
    comm.Ialltoall(a, r).Wait()
    assert r.tolist() == [me + 10 * q for q in range(p)]


def test_ialltoallv():
    comm, p, me = _world()
    sc = [q + 1 for q in range(p)]
    rc = [me + 1] * p
    s = torch.cat([torch.full((sc[q],), float(me)) for q in range(p)])
    r = torch.empty(sum(rc))
    req = comm.Ialltoallv((s, sc), (r, rc))
    req.Wait()
    assert torch.equal(r, torch.cat([torch.full((me + 1,), float(q)) for q in range(p)]))


def test_ibcast():
    comm, p, me = _world()
    t = torch.arange(5.0) * (me + 1)
    comm.Ibcast(t, root=0).Wait()
    assert torch.equal(t, torch.arange(5.0))


def test_iexscan():
    comm, p, me = _world()
    s = torch.tensor([2.0])
    out = torch.zeros(1)
    comm.Iexscan(s, out, MPI.SUM).Wait()
    if me:
        assert float(out) == 2.0 * me


def test_igather():
    comm, p, me = _world()
    t = torch.tensor([float(me)])
    out = torch.empty(p)
    comm.Igather(t, out, root=0).Wait()
    if me == 0:
        assert out.tolist() == list(map(float, range(p)))


def test_igatherv():
    comm, p, me = _world()
    counts, displs = _v(p)
    send = torch.full((counts[me],), float(me))
    out = torch.empty(sum(counts))
    comm.Igatherv(send, (out, counts, displs), root=p - 1).Wait()
    if me == p - 1:
        assert torch.equal(out, torch.cat([torch.full((c,), float(r)) for r, c in enumerate(counts)]))


def test_ireduce():
    comm, p, me = _world()
    t = torch.tensor([float(me + 1)])
    out = torch.zeros(1)
    comm.Ireduce(t, out, MPI.SUM, root=0).Wait()
    if me == 0:
        assert float(out) == p * (p + 1) / 2


def test_iscan():
    comm, p, me = _world()
    out = torch.zeros(1)
    comm.Iscan(torch.tensor([1.0]), out, MPI.SUM).Wait()
    assert float(out) == me + 1


def test_iscatter():
    comm, p, me = _world()
    src = torch.arange(2 * p, dtype=torch.float32).reshape(p, 2) if me == 0 else None
    out = torch.empty(1, 2)
    comm.Iscatter(src, out, root=0).Wait()
    assert out.tolist() == [[2.0 * me, 2.0 * me + 1]]


def test_iscatterv():
    comm, p, me = _world()
    counts, displs = _v(p)
    src = torch.cat([torch.full((c,), float(r)) for r, c in enumerate(counts)]) if me == 0 else None
    out = torch.empty(counts[me])
    comm.Iscatterv((src, counts, displs) if me == 0 else None, out, root=0).Wait()
    assert torch.all(out == me)


def test_mpi_in_place():
    comm, p, me = _world()
    t = torch.full((3,), float(me))
    comm.Allreduce(MPI.IN_PLACE, t, MPI.SUM)
    assert torch.all(t == p * (p - 1) / 2)
    counts = [2] * p
    displs = [2 * r for r in range(p)]
    recv = torch.zeros(2 * p)
    recv[2 * me: 2 * me + 2] = float(me)
    comm.Allgatherv(MPI.IN_PLACE, (recv, counts, displs))
    assert recv.tolist() == [float(r) for r in range(p) for _ in range(2)]


def test_reduce():
    comm, p, me = _world()
    t = torch.tensor([float(me), 1.0])
    out = torch.zeros(2)
    comm.Reduce(t, out, MPI.SUM, root=p - 1)
    if me == p - 1:
        assert out.tolist() == [p * (p - 1) / 2, float(p)]
    x = ht.full((3,), float(me + 1))
    y = ht.zeros((3,))
    comm.Reduce(x, y, MPI.MAX, root=0)
    if me == 0:
        assert torch.all(y.larray == p)


def test_scan():
    comm, p, me = _world()
    out = torch.zeros(2)
    comm.Scan(torch.tensor([1.0, float(me)]), out, MPI.SUM)
    assert out.tolist() == [float(me + 1), float(me * (me + 1) / 2)]
    comm.Scan(torch.tensor([float(me), -float(me)]), out, MPI.MAX)
    assert out.tolist() == [float(me), 0.0]


def test_scatter():
    comm, p, me = _world()
    src = torch.arange(3 * p, dtype=torch.float32).reshape(p, 3) if me == 0 else None
    out = torch.empty(1, 3)
    comm.Scatter(src, out, root=0)
    assert out.tolist() == [[3.0 * me, 3.0 * me + 1, 3.0 * me + 2]]
    assert comm.scatter([r * r for r in range(p)] if me == 0 else None, root=0) == me * me


def test_scatter_like_axes():
    comm, p, me = _world()
    data = torch.full((p, p), me, dtype=torch.int64)
    out = torch.zeros_like(data)
    comm.Alltoall(data, out, send_axis=0)
    assert torch.equal(out, torch.arange(p).reshape(-1, 1).repeat(1, p))
    comm.Alltoall(data, out, send_axis=1)
    assert torch.equal(out, torch.arange(p).reshape(1, -1).repeat(p, 1))
    # main send axis, minor receive axis
    data = torch.full((2 * p, 3), me, dtype=torch.int64)
    out = torch.zeros((2, 3 * p), dtype=torch.int64)
    comm.Alltoall(data, out, send_axis=0, recv_axis=1)
    assert torch.equal(out, torch.arange(p).repeat_interleave(3).reshape(1, -1).repeat(2, 1))


def test_scatterv():
    comm, p, me = _world()
    counts, displs = _v(p)
    src = torch.cat([torch.full((c, 2), float(r)) for r, c in enumerate(counts)]) if me == 0 else None
    out = torch.empty((counts[me], 2))
    comm.Scatterv((src, counts, displs) if me == 0 else None, out, root=0)
    assert torch.all(out == me)


def _sorted3d():
    return ht.array(np.arange(5 * 6 * 7, dtype=np.float32).reshape(5, 6, 7))


def test_allgathervSorting():
    comm, p, me = _world()
    full = _sorted3d().larray
    for ax in range(3):
        t = _sorted3d()
        t.resplit_(ax)
        counts, displs, _ = comm.counts_displs_shape(t.shape, ax)
        out = torch.empty(tuple(full.shape))
        comm.Allgatherv(t, (out, counts, displs), recv_axis=ax)
        assert torch.equal(out, full.cpu()), ax


def test_alltoallSorting():
    comm, p, me = _world()
    # split 2 -> split 1 by one Alltoallv along the receive / send axes
    src = _sorted3d()
    src.resplit_(2)
    ref = _sorted3d()
    ref.resplit_(1)
    out = torch.empty(ref.lshape)
    comm.Alltoallv(src.larray, out, send_axis=ref.split, recv_axis=src.split)
    assert torch.equal(out, ref.larray.cpu())
