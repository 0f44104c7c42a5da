"""Semantics pinned by the round-4 fast paths: ht.where's one-call path and its exact bitwise merge
(-0.0 and NaN survive), Python-number operands handed to torch directly (same result types and
values as the 0-d tensor path, integer overflow still raises), index shapes inferred on the meta device with bounds checks."""
import numpy as np
import pytest

import heat_amd as ht


@pytest.mark.parametrize("split_c,split_x,split_y", [(0, 0, 0), (None, 0, None), (0, None, 0), (None, None, None)])
def test_where_keeps_negative_zero_and_nan(split_c, split_x, split_y):
    x = np.array([1.0, -0.0, 3.0, np.nan, -0.0, 6.0], dtype=np.float32)
    y = np.array([-0.0, 2.0, -0.0, 4.0, 5.0, np.nan], dtype=np.float32)
    c = np.array([True, True, False, True, True, False])
    r = ht.where(ht.array(c, split=split_c), ht.array(x, split=split_x), ht.array(y, split=split_y)).numpy()
    ref = np.where(c, x, y)
    assert np.array_equal(r, ref, equal_nan=True)
    assert np.array_equal(np.signbit(r), np.signbit(ref))


def test_where_scalars_and_broadcast():
    c = np.array([[True, False, True], [False, False, True]])
    a = np.arange(6, dtype=np.float64).reshape(2, 3)
    assert np.array_equal(ht.where(ht.array(c, split=0), ht.array(a, split=0), -1.0).numpy(), np.where(c, a, -1.0))
    assert np.array_equal(ht.where(ht.array(c), 7, ht.array(a)).numpy(), np.where(c, 7, a))
    row = np.array([True, False, True])
    assert np.array_equal(ht.where(ht.array(row), ht.array(a, split=0), 0.5).numpy(), np.where(row, a, 0.5))


def test_number_operands_types_and_values():
    ai = ht.array(np.arange(-3, 5, dtype=np.int32), split=0)
    af = ht.array(np.linspace(-2, 2, 8, dtype=np.float32), split=0)
    n_i, n_f = ai.numpy(), af.numpy()
    assert (ai * 3).dtype == ht.int32 and np.array_equal((ai * 3).numpy(), n_i * 3)
    assert (ai + 2.5).dtype == ht.float32 and np.allclose((ai + 2.5).numpy(), n_i + 2.5)
    assert np.array_equal((ai > 1).numpy(), n_i > 1)
    assert np.allclose((af ** 2).numpy(), n_f ** 2)
    assert np.allclose((af - np.float64(0.25)).numpy(), n_f - 0.25)
    assert np.array_equal((ai // 2).numpy(), n_i // 2)
    assert np.array_equal((ai % 3).numpy(), n_i % 3)
    with pytest.raises(RuntimeError):
        ai + 2 ** 40             # does not fit int32: raised as before


def test_index_bounds_and_shapes():
    x = ht.arange(20, split=0).reshape((4, 5))
    assert x[ht.array([0, 3, -1])].gshape == (3, 5)
    assert x[:, ht.array([[0, 1], [4, 2]])].gshape == (4, 2, 2)
    assert x[np.array(1), 2].item() == 7
    with pytest.raises(IndexError):
        x[ht.array([4])]
    with pytest.raises(IndexError):
        x[:, ht.array([-6])]
    y = ht.zeros((10,))
    with pytest.raises(IndexError):
        y[ht.array([10])] = 1.0
    y[ht.array([1, 9])] = 2.0
    assert y.numpy()[[1, 9]].tolist() == [2.0, 2.0]
