"""Host (CPU) behaviour of the native-kernel entry points: the PyTorch reference paths that serve
host tensors and act as the numerics oracle of the GPU tests."""
import torch

from heat_amd import ops
from heat_amd.core.linalg import basics


def test_knn_topk_host_matches_bruteforce():
    g = torch.Generator().manual_seed(0)
    Q = torch.randn(50, 7, generator=g)
    T = torch.randn(300, 7, generator=g)
    d, i = ops.knn_topk(Q, T, 5)
    ref = torch.cdist(Q.double(), T.double()) ** 2
    rv, ri = ref.topk(5, largest=False)
    assert torch.allclose(d.double(), rv, rtol=1e-5, atol=1e-6)
    assert torch.equal(i, ri)
    # fewer training rows than k: padded with +inf / -1
    d, i = ops.knn_topk(Q, T[:3], 5)
    assert torch.all(i[:, 3:] == -1) and torch.all(torch.isinf(d[:, 3:]))


def test_gemm_split_host_is_plain_matmul():
    a, b = torch.randn(40, 30), torch.randn(30, 20)
    assert torch.allclose(ops.gemm_f16x3(a, b), a @ b)
    assert not basics._split_gemm_ok(a, b)   # host tensors never take the device split path


def test_small_k_pass_is_device_only():
    X, C = torch.randn(100, 8), torch.randn(4, 8)
    assert ops.kmeans_step_small(X, C) is None
    lab, mind = ops.kmeans_assign(X, C)
    d = torch.cdist(X.double(), C.double()) ** 2
    assert torch.equal(lab.long(), d.argmin(1))
    assert torch.allclose(mind.double(), d.min(1).values, rtol=1e-5, atol=1e-5)


def test_kmeans_update_host():
    X = torch.randn(500, 6)
    lab = torch.randint(0, 7, (500,), dtype=torch.int32)
    s, c = ops.kmeans_update(X, lab, 7)
    ref = torch.zeros(7, 6, dtype=torch.float64).index_add_(0, lab.long(), X.double())
    assert torch.allclose(s.double(), ref, atol=1e-4)
    assert torch.equal(c.long(), torch.bincount(lab.long(), minlength=7))
