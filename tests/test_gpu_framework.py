"""The whole CPU check suite again with the default device on the MI355X (world of one): every
factory, op, estimator and I/O path must keep its tensors on the GPU and agree with NumPy."""
import pytest

from . import dist_checks

pytestmark = pytest.mark.gpu

CHECKS = [n for n in dir(dist_checks) if n.startswith("check_")]


@pytest.mark.parametrize("name", CHECKS)
def test_on_gpu(name, gpu):
    getattr(dist_checks, name)()


def test_lasso_kernel_matches_host(gpu):
    import numpy as np
    import torch
    import heat_amd as ht

    rng = np.random.default_rng(0)
    X = rng.normal(size=(5000, 40)).astype(np.float32)
    X /= np.sqrt((X ** 2).mean(0))
    y = (X @ rng.normal(size=40).astype(np.float32)).astype(np.float32)
    th = []
    for dev in ("cpu", "gpu"):
        est = ht.regression.Lasso(lam=0.05, max_iter=30, tol=None)
        est.fit(ht.array(X, device=dev), ht.array(y[:, None], device=dev))
        th.append(est.theta.larray.cpu())
    assert torch.allclose(th[0], th[1], atol=2e-4), (th[0] - th[1]).abs().max()


def test_profiling_counts_native_kernels(gpu):
    import torch
    import heat_amd as ht
    from heat_amd import profiling

    profiling.reset()
    profiling.enable(timing=True)
    try:
        x = ht.random.randn(4096, 16, split=0)
        km = ht.cluster.KMeans(n_clusters=8, init="random", max_iter=3)    # fused small-k pass
        km.fit(x)
        km = ht.cluster.KMeans(n_clusters=40, init="random", max_iter=3)   # MFMA assign + update
        km.fit(x)
        c = profiling.counters()
    finally:
        profiling.disable()
    assert c["kmeans_step_small"]["calls"] >= 3 and c["kmeans_step_small"]["ms"] > 0
    assert c["kmeans_assign"]["calls"] >= 3 and c["kmeans_assign"]["ms"] > 0
    assert c["kmeans_update"]["calls"] >= 3


def test_data_parallel_on_gpu(gpu):
    """DataParallel + DataParallelOptimizer with a CUDA model (bucketed gradient hooks on the
    device); one rank: the step equals plain SGD."""
    import torch
    import heat_amd as ht

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4)).to(dev)
    opt = ht.optim.DataParallelOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), blocking=True)
    dp = ht.nn.DataParallel(net, ht.MPI_WORLD, opt, blocking_parameter_updates=True)
    ref = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4)).to(dev)
    ref.load_state_dict(net.state_dict())
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.1)
    x = torch.randn(64, 16, device=dev)
    y = torch.randint(0, 4, (64,), device=dev)
    for _ in range(3):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(dp(x), y).backward()
        opt.step()
        ref_opt.zero_grad()
        torch.nn.functional.cross_entropy(ref(x), y).backward()
        ref_opt.step()
    for p, q in zip(net.parameters(), ref.parameters()):
        assert torch.allclose(p, q, atol=1e-6)


def test_mnist_example_on_gpu(gpu):
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, os.path.join(root, "examples", "nn", "mnist.py"), "--epochs", "2",
                          "--samples", "2048"], capture_output=True, text=True, timeout=600, cwd=root)
    assert res.returncode == 0, res.stderr[-3000:]
    assert "epoch 1" in res.stdout


def test_debug_streams_detects_cross_stream_race(gpu):
    """HEAT_DEBUG_STREAMS=1: a collective issued on the default stream while a native kernel is
    still running on a side stream raises; after wait_stream it passes."""
    import torch

    import heat_amd as ht
    from heat_amd import ops

    old = ops.DEBUG_STREAMS
    ops.DEBUG_STREAMS = True
    try:
        side = torch.cuda.Stream()
        x = torch.randn(8192, 8192, device="cuda")
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            # ~5 ms of native kernels queued on the side stream (host enqueues far faster)
            for _ in range(100):
                ops.moments(x, None)
        raised = False
        try:
            ht.MPI_WORLD.Allreduce(ht.MPI.IN_PLACE, x[:1, :4].clone(), ht.MPI.SUM)
        except RuntimeError as e:
            raised = "stream-ordering race" in str(e)
        torch.cuda.current_stream().wait_stream(side)
        side.synchronize()
        ht.MPI_WORLD.Allreduce(ht.MPI.IN_PLACE, x[:1, :4].clone(), ht.MPI.SUM)
        assert raised
    finally:
        ops.DEBUG_STREAMS = old
        ops.LAST_LAUNCH_STREAM.clear()


def test_kmeans_graph_replay_matches_eager(gpu):
    """HEAT_KMEANS_GRAPH=1: the Lloyd step replayed from a captured HIP graph gives the same
    centroids as eager launches. Runs in a child process started with
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 (read at HIP init; graph mode requires it, see
    ``KMeans._graph_ok``)."""
    import os
    import subprocess
    import sys

    code = """
import os, torch, heat_amd as ht
ht.use_device("gpu")
ht.random.seed(5)
x = ht.random.randn(200_000, 64, split=0)
X = x.larray
os.environ["HEAT_KMEANS_GRAPH"] = "1"
km = ht.cluster.KMeans(n_clusters=256, init="random", max_iter=1, tol=None, random_state=1)
km.step(x)   # packs the points (and re-arms the certified probe): always eager
km._certify, km._cert_probe = False, None
worst = []
for _ in range(5):
    C = km.cluster_centers_.larray.clone()
    eager, _ = km._centroid_step(X, C, x.comm, False)   # the same step, launched eagerly
    eager = eager.clone()
    km.step(x)   # replayed from the graph
    torch.cuda.synchronize()
    d = (km.cluster_centers_.larray - eager).abs()
    worst.append((float(d.median()), float(d.max())))
assert getattr(km, "_graph", None) is not None
# per step: identical labels, sums within float-atomic rounding
assert all(m < 1e-5 and M < 1e-3 for m, M in worst), worst
print("OK", worst)
"""
    env = dict(os.environ, DEBUG_CLR_GRAPH_PACKET_CAPTURE="0", HEAT_KMEANS_GRAPH="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=110,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_scalar_division_and_pow_exact_on_device(gpu):
    """Division and pow by a Python number on a device array are correctly rounded (the 0-d
    tensor path; torch's scalar form multiplies by the reciprocal): bitwise equal to NumPy."""
    import numpy as np
    import heat_amd as ht

    rng = np.random.default_rng(3)
    x = rng.normal(size=4099).astype(np.float32) * 1e3
    a = ht.array(x, split=0, device="gpu")
    assert a.larray.is_cuda
    for v in (3.0, 7.0, 1e-40, 0.1):
        got = (a / v).numpy()
        ref = (x / np.float32(v)).astype(np.float32)
        assert np.array_equal(got, ref), v
    assert np.all(np.isfinite((a / 1e-40).numpy()[np.abs(x) < 1e-3]))
    np.testing.assert_allclose((a ** 3.0).numpy(), np.power(x.astype(np.float64), 3.0), rtol=3e-7)
