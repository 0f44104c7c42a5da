"""Native stable radix sort (``ops/csrc/radix.hip``) against ``torch.sort(stable=True)`` on the
device: float32 / int32, ascending and descending, single rows and batches (row-number digit
passes), ragged tiles, NaN / +-0.0 / duplicates; and ``ht.sort`` using it."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from heat_amd import ops

    assert ops.available(), "native library must load on a GPU box"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("shape", [(1,), (4095,), (4097,), (1000003,), (3, 5000), (300, 777), (70000, 3), (2, 1)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.int32])
@pytest.mark.parametrize("descending", [False, True])
def test_radix_sort_matches_torch(shape, dtype, descending):
    from heat_amd import ops

    dev = _dev()
    g = torch.Generator().manual_seed(sum(shape))
    if dtype == torch.float32:
        x = torch.randn(shape, generator=g)
        x = torch.round(x * 8) / 8  # many ties
    else:
        x = torch.randint(-50, 50, shape, generator=g, dtype=torch.int32)
    xd = x.to(dev)
    v, i = ops.sort_rows(xd, descending)
    rv, ri = torch.sort(xd, dim=-1, descending=descending, stable=True)
    assert torch.equal(v, rv)
    assert torch.equal(i, ri)


def test_radix_sort_special_values():
    from heat_amd import ops

    dev = _dev()
    x = torch.tensor([1.0, float("nan"), -0.0, 0.0, -float("inf"), float("inf"), -0.0, float("nan"), 2.0, -1.0] * 1000)
    xd = x.to(dev)
    for desc in (False, True):
        v, i = ops.sort_rows(xd, desc)
        rv, ri = torch.sort(xd, descending=desc, stable=True)
        assert torch.equal(i, ri)
        assert torch.equal(torch.isnan(v), torch.isnan(rv))
        ok = ~torch.isnan(rv)
        assert torch.equal(v[ok], rv[ok])
        # -0.0 kept bit-exact (values are gathered, not reconstructed)
        assert torch.equal(torch.signbit(v[ok]), torch.signbit(rv[ok]))


def test_ht_sort_uses_radix(gpu):
    import heat_amd as ht
    from heat_amd import ops

    assert ops.radix_sort_supported(torch.zeros(5000, 16, device="cuda"), 0)
    assert ops.radix_sort_supported(torch.zeros(16, 5000, device="cuda"), 1)

    a = np.random.default_rng(3).standard_normal((5000, 7)).astype(np.float32)
    for axis in (0, 1):
        for split in (None, 0, 1):
            x = ht.array(a, split=split)
            v, i = ht.sort(x, axis=axis)
            assert np.array_equal(v.numpy(), np.sort(a, axis=axis, kind="stable"))
            assert np.array_equal(i.numpy(), np.argsort(a, axis=axis, kind="stable"))
