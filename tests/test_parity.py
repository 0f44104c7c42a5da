"""Reference-parity checks (``tests/parity/*_checks.py``, one module per reference test file,
one check per reference test method): each runs in a world of one (in-process, one pytest case
per check) and, batched per module, in 2, 3, 5 and 8 gloo ranks."""
import importlib
import os

import pytest

from ._dist import run_distributed, run_distributed_batch

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "parity")
MODULES = sorted("tests.parity." + f[:-3] for f in os.listdir(HERE) if f.endswith("_checks.py"))
CASES = []
for _m in MODULES:
    _mod = importlib.import_module(_m)
    CASES += [(_m, n) for n in sorted(dir(_mod)) if n.startswith("test_") and callable(getattr(_mod, n))]
_BATCH = {}


def _ids(case):
    return "{}::{}".format(case[0].rsplit(".", 1)[1].replace("_checks", ""), case[1])


@pytest.mark.parametrize("module,name", CASES, ids=[_ids(c) for c in CASES])
def test_parity_local(module, name):
    getattr(importlib.import_module(module), name)()


@pytest.mark.parametrize("nprocs", [2, 3, 5, 8])
@pytest.mark.parametrize("module,name", CASES, ids=[_ids(c) for c in CASES])
def test_parity_distributed(module, name, nprocs):
    key = (module, nprocs)
    if key not in _BATCH:
        _BATCH[key] = run_distributed_batch(module, [n for m, n in CASES if m == module], nprocs)
    ok, err = _BATCH[key][name]
    if not ok:
        run_distributed(module + ":" + name, nprocs)
        pytest.fail("check {} failed in the batched job but passed alone:\n{}".format(name, err))
