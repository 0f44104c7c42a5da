"""Parity with ``heat/core/tests/test_suites/test_basic_test.py``: the downstream test base class
``heat_amd.testing.TestCase`` (local-block and global array comparison, function-vs-numpy sweeps
over every split axis, memory-layout assertion)."""
import numpy as np
import torch

import heat_amd as ht
from heat_amd.testing import TestCase

from ._util import raises


def _case():
    tc = TestCase("__init__")
    tc.device = ht.get_device()
    return tc


def test_assert_array_equal():
    tc = _case()
    p = tc.get_size()
    a = ht.ones((p, 10, 10), dtype=ht.int32, split=1)
    e = np.ones((p, 10, 10), dtype=np.int32)
    tc.assert_array_equal(a, e)
    e[0, 1, 1] = 0
    raises(AssertionError, tc.assert_array_equal, a, e)
    z = ht.zeros((25, 13, p, 20), dtype=ht.float32, split=2)
    tc.assert_array_equal(z, torch.zeros((25, 13, p, 20), dtype=torch.float32, device=z.device.torch_device))
    # everything on rank 0: balanced before the local comparison
    dev = tc.device.torch_device
    data = torch.arange(p, dtype=torch.int32, device=dev) if tc.get_rank() == 0 else \
        torch.empty((0,), dtype=torch.int32, device=dev)
    tc.assert_array_equal(ht.array(data, is_split=0), np.arange(p, dtype=np.int32))
    # a wrong global shape and a non-array expectation are assertion failures
    raises(AssertionError, tc.assert_array_equal, a, np.ones((p, 10, 9), dtype=np.int32))
    raises(AssertionError, tc.assert_array_equal, a, [1, 2])
    raises(AssertionError, tc.assert_array_equal, np.ones(3), np.ones(3))


def test_assert_func_equal():
    tc = _case()
    shape = (5, 3, 2, 9)
    tc.assert_func_equal(shape, heat_func=ht.exp, numpy_func=np.exp, low=-10, high=10)
    tc.assert_func_equal(shape, heat_func=ht.exp2, numpy_func=np.exp2, low=-10, high=10)
    tc.assert_func_equal(shape, heat_func=ht.log, numpy_func=np.log, data_types=[np.int32, np.int64], low=1)
    raises(AssertionError, tc.assert_func_equal, shape, heat_func=ht.exp, numpy_func=np.exp2, low=-10, high=10)
    raises(ValueError, tc.assert_func_equal, np.ones(shape), heat_func=np.exp, numpy_func=np.exp)
    raises(ValueError, tc.assert_func_equal, shape, heat_func=ht.exp, numpy_func=np.exp, low=-100, high=100,
           data_types=[object])


def test_assert_func_equal_for_tensor():
    tc = _case()
    tc.assert_func_equal_for_tensor(np.ones((tc.get_size(), 20), dtype=np.int8), ht.any, np.any,
                                    distributed_result=False)
    arr = np.array([[1, 2, 4, 1, 3], [1, 4, 7, 5, 1]], dtype=np.int8)
    tc.assert_func_equal_for_tensor(arr, ht.expand_dims, np.expand_dims, heat_args={"axis": 1},
                                    numpy_args={"axis": 1})
    torch.manual_seed(3)   # the same tensor on every rank
    t = torch.randn(15, 15).to(tc.device.torch_device)
    tc.assert_func_equal_for_tensor(t, heat_func=ht.exp, numpy_func=np.exp)
    raises(TypeError, tc.assert_func_equal_for_tensor, ht.ones((15, 15)), heat_func=ht.exp, numpy_func=np.exp)


def test_assertTrue_memory_layout():
    tc = _case()
    data = torch.arange(3 * 4 * 5).reshape(3, 4, 5)
    a_c = ht.array(data)
    a_f = ht.array(data, order="F")
    tc.assertTrue_memory_layout(a_c, "C")
    tc.assertTrue_memory_layout(a_f, "F")
    raises(AssertionError, tc.assertTrue_memory_layout, a_c, "F")
    raises(ValueError, tc.assertTrue_memory_layout, a_f, order="K")
