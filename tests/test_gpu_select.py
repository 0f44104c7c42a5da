"""Packed-key arg-reduction and per-row top-k kernels (``ops/csrc/select.hip``) against NumPy /
PyTorch references on the device: all dtypes the kernels take, every axis, ties (first index),
NaN semantics (NumPy argmax/argmin: first NaN; torch.topk: NaN is the largest value)."""
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


DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.int32, torch.int16, torch.int8, torch.uint8]


def _data(shape, dtype, seed, ties=False):
    g = torch.Generator().manual_seed(seed)
    if dtype.is_floating_point:
        x = torch.randn(shape, generator=g)
        if ties:
            x = torch.round(x * 2) / 2
        return x.to(dtype)
    lo, hi = (0, 200) if dtype == torch.uint8 else (-100, 100)
    if ties:
        lo, hi = lo // 20, hi // 20
    return torch.randint(lo, hi, shape, generator=g).to(dtype)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(1000003,), (257, 1031), (33, 17, 65), (4, 100000), (100000, 3)])
@pytest.mark.parametrize("ties", [False, True])
def test_argreduce_keys(dtype, shape, ties):
    from heat_amd import ops

    dev = _dev()
    x = _data(shape, dtype, seed=sum(shape), ties=ties)
    xn = x.float().numpy() if dtype == torch.bfloat16 else x.numpy()
    xd = x.to(dev)
    for smallest in (False, True):
        ref_fn = np.argmin if smallest else np.argmax
        k = ops.argreduce_keys(xd, None, smallest)
        assert int(ops.argreduce_decode(k)) == int(ref_fn(xn.reshape(-1)))
        for ax in range(len(shape)):
            k = ops.argreduce_keys(xd, ax, smallest)
            got = ops.argreduce_decode(k).cpu().numpy()
            assert np.array_equal(got, ref_fn(xn, axis=ax)), (ax, smallest)


def test_argreduce_nan_and_split_offsets():
    """NaN wins both argmax and argmin (first NaN, NumPy); axis=None on a block of a split array
    returns the GLOBAL flat index."""
    from heat_amd import ops

    dev = _dev()
    x = torch.randn(50, 40)
    x[7, 3] = float("nan")
    x[20, 1] = float("nan")
    for smallest in (False, True):
        k = ops.argreduce_keys(x.to(dev), None, smallest)
        assert int(ops.argreduce_decode(k)) == 7 * 40 + 3
        k = ops.argreduce_keys(x.to(dev), 0, smallest)
        ref = (np.argmin if smallest else np.argmax)(x.numpy(), axis=0)
        assert np.array_equal(ops.argreduce_decode(k).cpu().numpy(), ref)
    # rows 10..29 of a (100, 40) array split along axis 0: global flat index
    full = torch.randn(100, 40)
    blk = full[10:30].contiguous().to(dev)
    k = ops.argreduce_keys(blk, None, False, displ=10, gextent=100, split=0)
    assert int(ops.argreduce_decode(k)) == int(np.argmax(full[10:30].numpy())) + 10 * 40
    # columns 5..19 of a split=1 array
    blk = full[:, 5:20].contiguous().to(dev)
    k = ops.argreduce_keys(blk, None, True, displ=5, gextent=40, split=1)
    r, c = np.unravel_index(int(np.argmin(full[:, 5:20].numpy())), (100, 15))
    assert int(ops.argreduce_decode(k)) == r * 40 + c + 5


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16, torch.int32, torch.int8])
@pytest.mark.parametrize("shape,dim", [((1000, 777), 1), ((1000, 777), 0), ((5, 100003), -1), ((64, 9, 33), 1)])
@pytest.mark.parametrize("k", [1, 3, 8, 16, 32])
@pytest.mark.parametrize("largest", [True, False])
def test_topk_rows(dtype, shape, dim, k, largest):
    from heat_amd import ops

    dev = _dev()
    if shape[dim] < k:
        pytest.skip("k larger than the row")
    x = _data(shape, dtype, seed=k + sum(shape), ties=dtype in (torch.int8,)).to(dev)
    res = ops.topk_rows(x, k, dim, largest)
    assert res is not None
    v, i = res
    rv, _ = torch.topk(x.float(), k, dim=dim, largest=largest, sorted=True)
    assert torch.equal(v.float(), rv)
    assert torch.equal(torch.gather(x, dim, i), v)
    # ties resolve to the smaller index: within equal values the indices ascend
    vv, ii = v.movedim(dim, -1).float(), i.movedim(dim, -1)
    same = vv[..., 1:] == vv[..., :-1]
    assert torch.all(~same | (ii[..., 1:] > ii[..., :-1]))


def test_topk_nan_like_torch():
    from heat_amd import ops

    dev = _dev()
    x = torch.randn(300, 50)
    x[::7, 3] = float("nan")
    xd = x.to(dev)
    v, i = ops.topk_rows(xd, 4, 1, True)
    assert torch.isnan(v[::7, 0]).all()            # NaN is the largest value
    v, i = ops.topk_rows(xd, 4, 1, False)
    assert not torch.isnan(v).any()                 # ... and so never among the smallest
    rv, _ = torch.topk(xd, 4, dim=1, largest=False)
    assert torch.equal(v, rv)


def test_ht_argmax_topk_use_kernels(gpu):
    import heat_amd as ht

    x = ht.random.randn(1000, 300, split=0)
    xn = x.numpy()
    assert int(ht.argmax(x).item()) == int(np.argmax(xn))
    assert np.array_equal(ht.argmin(x, axis=0).numpy(), np.argmin(xn, axis=0))
    assert np.array_equal(ht.argmax(x, axis=1).numpy(), np.argmax(xn, axis=1))
    v, i = ht.topk(x, 5, dim=1)
    rv, _ = torch.topk(torch.from_numpy(xn), 5, dim=1)
    assert np.array_equal(v.numpy(), rv.numpy())
    v, i = ht.topk(x, 5, dim=0, largest=False)
    rv, _ = torch.topk(torch.from_numpy(xn), 5, dim=0, largest=False)
    assert np.array_equal(v.numpy(), rv.numpy())
