"""Native stream-ordered RCCL communicator (``ops/csrc/comm.hip``, ``parallel/native_comm.py``) in a
world of one on the MI355X: it binds torch's RCCL instance, initialises a communicator, and every
collective runs on the caller's stream with the expected result (identity at one rank); the
exchange path of ``exchange_axis`` moves raw bytes of any dtype."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_native_comm_world_of_one(gpu):
    import heat_amd as ht
    from heat_amd.parallel import native_comm

    assert native_comm.rccl_path() is not None
    nc = native_comm.NativeComm(ht.MPI_WORLD)
    try:
        x = torch.arange(1000, dtype=torch.float32, device="cuda")
        for op in ("sum", "max", "min", "prod"):
            y = x.clone()
            nc.allreduce_(y, op)
            torch.cuda.synchronize()
            assert torch.equal(y, x), op
        for dt in (torch.float64, torch.int32, torch.int64, torch.bfloat16, torch.uint8):
            y = x.to(dt)
            assert torch.equal(nc.allreduce_(y.clone(), "sum"), y)
        g = nc.allgather(x.reshape(10, 100))
        assert g.shape == (1, 10, 100) and torch.equal(g[0], x.reshape(10, 100))
        b = x.clone()
        assert torch.equal(nc.broadcast_(b, 0), x)
        src = torch.randint(0, 255, (4096,), dtype=torch.uint8, device="cuda")
        dst = torch.empty_like(src)
        nc.alltoallv_bytes(src, [4096], dst, [4096])
        torch.cuda.synchronize()
        assert torch.equal(dst, src)
        # stream ordering: the collective follows the kernel queued before it on the same stream
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            z = torch.full((1 << 20,), 3.0, device="cuda")
            z.mul_(2.0)
            nc.allreduce_(z, "sum")
            z.add_(1.0)
        s.synchronize()
        assert bool((z == 7.0).all())
        nc.check()
    finally:
        nc.close()
