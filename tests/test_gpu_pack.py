"""Native block pack/unpack (``csrc/pack.hip``) against the torch reference (narrow + cat) for
every axis, uneven and empty blocks, every word width (odd byte rows down to 1-byte words) and
dtypes; the round trip is exact."""
import numpy as np
import pytest
import torch

from heat_amd import ops

pytestmark = pytest.mark.gpu


def _ref_pack(t, axis, counts):
    off = np.concatenate([[0], np.cumsum(counts)]).astype(int)
    return torch.cat([t.narrow(axis, int(off[q]), int(c)).reshape(-1) for q, c in enumerate(counts)])


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int16, torch.uint8, torch.bool,
                                   torch.complex64])
@pytest.mark.parametrize("shape,axis,counts", [((37, 5, 3), 0, [10, 0, 27]), ((4, 29, 7), 1, [3, 9, 0, 17]),
                                               ((6, 5, 11), 2, [1, 1, 9]), ((1000,), 0, [250, 250, 250, 250]),
                                               ((3, 8, 16), 1, [2] * 4), ((2, 3), 1, [3])])
def test_pack_roundtrip(gpu, dtype, shape, axis, counts):
    assert ops.pack_supported(torch.zeros(1, device="cuda"))
    g = torch.Generator().manual_seed(3)
    base = torch.randint(0, 100, shape, generator=g)
    t = (base % 2 == 0) if dtype == torch.bool else base.to(dtype)
    t = t.cuda()
    packed = ops.pack_blocks(t, axis, counts)
    ref = _ref_pack(t, axis, counts)
    assert packed.shape == ref.shape and torch.equal(packed, ref)
    back = ops.unpack_blocks(packed, t.shape, axis, counts)
    assert torch.equal(back, t)


def test_pack_large_many_blocks(gpu):
    t = torch.randn(64, 4096, 33, device="cuda")
    counts = [4096 // 256] * 256
    p = ops.pack_blocks(t, 1, counts)
    assert torch.equal(p, _ref_pack(t, 1, counts))
    assert torch.equal(ops.unpack_blocks(p, t.shape, 1, counts), t)
