"""Parity with ``heat/core/tests/test_printing.py``: print-option profiles and setters, and the
exact ``DNDarray(...)`` text of empty, scalar, unbalanced, replicated and split arrays below and
above the summarisation threshold. Expected strings are built from torch's formatter on the
gathered data with the same options (the format the reference prints), re-indented for the
``DNDarray(`` prefix - independent of the distributed gather under test."""
import math

import numpy as np
import torch

import heat_amd as ht

from ._util import raises

DEFAULTS = {"precision": 4, "threshold": 1000, "edgeitems": 3, "linewidth": 120, "sci_mode": None}


def _expected(data: np.ndarray, dtype: str, split, **opts):
    o = dict(DEFAULTS)
    o.update(opts)
    saved = ht.get_printoptions()
    torch.set_printoptions(precision=o["precision"], threshold=o["threshold"], edgeitems=o["edgeitems"],
                           linewidth=o["linewidth"], sci_mode=o["sci_mode"])
    try:
        body = str(torch.as_tensor(data))
    finally:
        torch.set_printoptions(profile="default")
        ht.set_printoptions(**saved)
    # torch's suffix (dtype=...) is dropped; continuation lines move right by len("DNDarray(") - len("tensor(")
    body = body[len("tensor("):]
    if body.endswith(")"):
        body = body[:-1]
    for suffix in (", dtype=torch.float64", ", dtype=torch.int32", ", dtype=torch.int64", ", dtype=torch.float32"):
        if body.endswith(suffix):
            body = body[: -len(suffix)]
    body = body.replace("\n       ", "\n         ").replace("\n\n         ", "\n\n         ")
    return "DNDarray({}, dtype=ht.{}, device=cpu:0, split={})".format(body, dtype, split)


def _with(opts, fn):
    ht.set_printoptions(**opts)
    try:
        fn()
    finally:
        ht.set_printoptions(profile="default")


def test_get_default_options():
    assert ht.get_printoptions() == DEFAULTS


def test_set_get_short_options():
    _with({"profile": "short"}, lambda: ht.get_printoptions() == dict(DEFAULTS, precision=2, edgeitems=2) or
          (_ for _ in ()).throw(AssertionError(ht.get_printoptions())))


def test_set_get_full_options():
    def chk():
        assert ht.get_printoptions() == dict(DEFAULTS, threshold=math.inf), ht.get_printoptions()
    _with({"profile": "full"}, chk)


def test_set_get_precision():
    _with({"precision": 6}, lambda: None if ht.get_printoptions()["precision"] == 6 else 1 / 0)


def test_set_get_threshold():
    _with({"threshold": 7}, lambda: None if ht.get_printoptions()["threshold"] == 7 else 1 / 0)


def test_set_get_edgeitems():
    _with({"edgeitems": 8}, lambda: None if ht.get_printoptions()["edgeitems"] == 8 else 1 / 0)


def test_set_get_linewidth():
    _with({"linewidth": 9}, lambda: None if ht.get_printoptions()["linewidth"] == 9 else 1 / 0)


def test_set_get_sci_mode():
    _with({"sci_mode": True}, lambda: None if ht.get_printoptions()["sci_mode"] is True else 1 / 0)


def _check(x, expected):
    s = str(x)
    if x.comm.rank == 0:
        assert s == expected, "\n{}\n!=\n{}".format(s, expected)


def test_empty():
    _check(ht.array([], dtype=ht.int64), "DNDarray([], dtype=ht.int64, device=cpu:0, split=None)")


def test_scalar():
    _check(ht.array(42), "DNDarray(42, dtype=ht.int64, device=cpu:0, split=None)")


def test_unbalanced():
    d = ht.arange(2 * 3 * 4, split=0).reshape((2, 3, 4))
    _check(d[0], _expected(np.arange(12, dtype=np.int32).reshape(3, 4), "int32", d[0].split))


def test_unsplit_below_threshold():
    _check(ht.arange(24).reshape((2, 3, 4)), _expected(np.arange(24, dtype=np.int32).reshape(2, 3, 4), "int32", None))


def test_unsplit_above_threshold():
    n = np.arange(12 * 13 * 14, dtype=np.int32).reshape(12, 13, 14)
    _check(ht.arange(12 * 13 * 14).reshape((12, 13, 14)), _expected(n, "int32", None))


def _split_case(shape, split, opts, dtype=np.float32, start=0.5):
    def run():
        n = (np.arange(int(np.prod(shape)), dtype=np.float64) + start).astype(dtype).reshape(shape)
        x = ht.array(n, split=split)
        _check(x, _expected(n, "float32" if dtype == np.float32 else "float64", split, **opts))
    _with(opts, run)


def test_split_0_below_threshold():
    _split_case((2, 3, 4), 0, {"precision": 2})


def test_split_0_above_threshold():
    _split_case((10, 11, 12), 0, {"precision": 1}, start=0.2)


def test_split_1_below_threshold():
    _split_case((4, 5, 6), 1, {"sci_mode": True}, dtype=np.float64)


def test_split_1_above_threshold():
    _split_case((10, 11, 12), 1, {"edgeitems": 2}, start=0.2)


def test_split_2_below_threshold():
    _split_case((2, 3, 4), 2, {"linewidth": 40})


def test_split_2_above_threshold():
    _split_case((10, 11, 12), 2, {"precision": 6, "edgeitems": 2, "linewidth": 160}, dtype=np.float64, start=0.2)

