"""Helpers shared by the parity checks (world-size independent)."""
from __future__ import annotations

import numpy as np
import torch

import heat_amd as ht

from ..dist_checks import assert_array_equal  # noqa: F401


def splits(ndim: int):
    return [None] + list(range(ndim))


def raises(exc, fn, *args, **kwargs):
    try:
        fn(*args, **kwargs)
    except exc:
        return
    except Exception as e:  # noqa: B902 - reported
        raise AssertionError("{} raised {} instead of {}".format(getattr(fn, "__name__", fn), type(e).__name__, exc))
    raise AssertionError("{} did not raise {}".format(getattr(fn, "__name__", fn), exc))


def close(a, expected, rtol=1e-5, atol=1e-6):
    got = a.numpy() if isinstance(a, ht.DNDarray) else np.asarray(a)
    expected = np.asarray(expected)
    assert got.shape == expected.shape, "shape {} != {}".format(got.shape, expected.shape)
    assert np.allclose(got, expected, rtol=rtol, atol=atol, equal_nan=True), "{}\n!=\n{}".format(got, expected)


def same(a, expected):
    got = a.numpy() if isinstance(a, ht.DNDarray) else np.asarray(a)
    expected = np.asarray(expected)
    assert got.shape == expected.shape, "shape {} != {}".format(got.shape, expected.shape)
    assert np.array_equal(got, expected), "{}\n!=\n{}".format(got, expected)


def rng(seed=0):
    return np.random.default_rng(seed)


def each_split(data, fn):
    """fn(DNDarray, split) for every split of ``data`` (NumPy array)."""
    for s in splits(np.ndim(data)):
        fn(ht.array(data, split=s), s)
