"""
Test-suite base class for code built on heat_amd (reference ``heat/core/tests/test_suites/basic_test.py``:
``TestCase`` 12, ``assert_array_equal`` 68, ``assert_func_equal`` 142,
``assert_func_equal_for_tensor`` 219, ``assertTrue_memory_layout`` 308).

Downstream projects subclass :class:`TestCase` and compare distributed results against numpy:

* :meth:`TestCase.assert_array_equal` checks the global shape, then every rank's LOCAL block
  against the matching slice of the expected array (so a wrong distribution fails even when the
  gathered values happen to match), then the gathered values.
* :meth:`TestCase.assert_func_equal` / :meth:`assert_func_equal_for_tensor` run a heat function
  on random data split along every axis in turn and compare with the numpy equivalent.

The device comes from ``HEAT_TEST_USE_DEVICE`` (``cpu`` default, or ``gpu``).
"""
from __future__ import annotations

import os
import unittest
from typing import Callable, Optional, Sequence

import numpy as np
import torch

from . import core as ht
from .core.dndarray import DNDarray

__all__ = ["TestCase"]


class TestCase(unittest.TestCase):
    """``unittest.TestCase`` with distributed-array assertions."""

    device = None
    other_device = None
    envar = None

    @property
    def comm(self):
        return ht.get_comm()

    @classmethod
    def setUpClass(cls):
        envar = os.getenv("HEAT_TEST_USE_DEVICE", "cpu")
        if envar == "cpu":
            ht.use_device("cpu")
            cls.device, cls.other_device = ht.cpu, ht.cpu
            if torch.cuda.is_available():
                cls.other_device = ht.gpu
        elif envar == "gpu" and torch.cuda.is_available():
            ht.use_device("gpu")
            torch.cuda.set_device(torch.device(ht.gpu.torch_device))
            cls.device, cls.other_device = ht.gpu, ht.cpu
        else:
            raise RuntimeError("Value '{}' of environment variable 'HEAT_TEST_USE_DEVICE' is unsupported"
                               .format(envar))
        cls.envar = envar

    def _device(self):
        return self.device if self.device is not None else ht.get_device()

    def get_rank(self) -> int:
        return self.comm.rank

    def get_size(self) -> int:
        return self.comm.size

    # ------------------------------------------------------------------ array comparison
    def assert_array_equal(self, heat_array: DNDarray, expected_array) -> None:
        """``heat_array`` equals ``expected_array`` (numpy array or torch tensor) globally AND in
        every rank's local block (an unbalanced array is balanced first)."""
        if isinstance(expected_array, torch.Tensor):
            expected_array = expected_array.detach().cpu().numpy()
        self.assertIsInstance(heat_array, DNDarray,
                              "The array to test was not a ht.DNDarray but {}".format(type(heat_array)))
        self.assertIsInstance(expected_array, np.ndarray,
                              "The expected array was not a numpy.ndarray or torch.Tensor but {}"
                              .format(type(expected_array)))
        self.assertEqual(tuple(heat_array.shape), tuple(expected_array.shape),
                         "Global shapes do not match: {} vs expected {}".format(heat_array.shape,
                                                                              expected_array.shape))
        if not heat_array.is_balanced():
            heat_array.balance_()
        _, _, sl = heat_array.comm.chunk(heat_array.gshape, heat_array.split)
        local_expected = expected_array[sl]
        # 0 ok, 1 local values differ, 2 local shape differs; agreed on by every rank before any
        # rank raises (a lone raise would leave the others waiting in the gather below)
        code = 2 if tuple(heat_array.lshape) != tuple(local_expected.shape) else \
            0 if np.allclose(heat_array.larray.detach().cpu().numpy(), local_expected) else 1
        if heat_array.comm.size > 1:
            code = heat_array.comm.allreduce(code, ht.MPI.MAX)
        self.assertNotEqual(code, 2, "Local shapes do not match on some rank (here {} vs expected {})".format(
            heat_array.lshape, local_expected.shape))
        self.assertEqual(code, 0, "a local block differs from the expected slice")
        self.assertTrue(np.allclose(heat_array.numpy(), expected_array), "gathered array differs")

    def assert_func_equal(self, shape, heat_func: Callable, numpy_func: Callable, distributed_result: bool = True,
                          heat_args: Optional[dict] = None, numpy_args: Optional[dict] = None,
                          data_types: Sequence = (np.int32, np.int64, np.float32, np.float64), low: int = -10000,
                          high: int = 10000) -> None:
        """Random arrays of ``shape`` in each of ``data_types`` through
        :meth:`assert_func_equal_for_tensor`."""
        if not isinstance(shape, (tuple, list)):
            raise ValueError("The shape must be either a list or a tuple but was {}".format(type(shape)))
        for dt in data_types:
            self.assert_func_equal_for_tensor(self._random_array(shape, dt, low, high), heat_func, numpy_func,
                                              heat_args=heat_args, numpy_args=numpy_args,
                                              distributed_result=distributed_result)

    def assert_func_equal_for_tensor(self, tensor, heat_func: Callable, numpy_func: Callable,
                                     heat_args: Optional[dict] = None, numpy_args: Optional[dict] = None,
                                     distributed_result: bool = True) -> None:
        """``heat_func`` on ``tensor`` split along each axis in turn equals ``numpy_func`` on it;
        with ``distributed_result=False`` every rank must hold the full result."""
        self.assertTrue(callable(heat_func))
        self.assertTrue(callable(numpy_func))
        heat_args = heat_args or {}
        numpy_args = numpy_args or {}
        dev = self._device()
        if isinstance(tensor, np.ndarray):
            np_in = tensor
            t = torch.from_numpy(tensor.copy()).to(dev.torch_device)
        elif isinstance(tensor, torch.Tensor):
            t = tensor
            np_in = tensor.detach().cpu().numpy().copy()
        else:
            raise TypeError("The input tensors type must be one of [tuple, list, numpy.ndarray, torch.tensor] "
                            "but is {}".format(type(tensor)))
        expected = numpy_func(np_in, **numpy_args)
        if not isinstance(expected, np.ndarray):
            expected = np.array([expected])
        dtype = ht.types.canonical_heat_type(t.dtype)
        for axis in range(t.dim()):
            a = ht.array(t, split=axis, dtype=dtype, device=dev, comm=self.comm)
            res = heat_func(a, **heat_args)
            self.assertEqual(a.device, res.device)
            self.assertEqual(a.larray.device, res.larray.device)
            if distributed_result:
                self.assert_array_equal(res, expected)
            else:
                self.assertTrue(np.array_equal(res.larray.detach().cpu().numpy(), expected))

    def assertTrue_memory_layout(self, tensor: DNDarray, order: str) -> None:  # noqa: N802 (reference name)
        """The local tensor's strides are row-major (``order='C'``) or column-major (``'F'``)."""
        strides = np.asarray(tensor.larray.stride())
        if order == "C":
            return self.assertTrue(bool(np.all(np.diff(strides) <= 0)))
        if order == "F":
            return self.assertTrue(bool(np.all(np.diff(strides) >= 0)))
        raise ValueError("expected order to be 'C' or 'F', but was {}".format(order))

    # ------------------------------------------------------------------ helpers
    def _random_array(self, shape, dtype, low: int, high: int) -> np.ndarray:
        """Random array, identical on every rank (the seed is drawn on rank 0 and broadcast)."""
        seed = self.comm.bcast(int(np.random.randint(1_000_000)), root=0)
        gen = np.random.default_rng(seed)
        if isinstance(dtype, type) and issubclass(dtype, np.floating):
            return gen.standard_normal(tuple(shape)).astype(dtype)
        if isinstance(dtype, type) and issubclass(dtype, np.integer):
            return gen.integers(low, high, size=tuple(shape)).astype(dtype)
        raise ValueError("Unsupported dtype. Expected a subclass of `np.floating` or `np.integer` but got {}"
                         .format(dtype))
