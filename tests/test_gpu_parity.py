"""The reference-parity checks (``tests/parity``) again with the default device on the MI355X
(world of one): factories, element-wise ops, reductions, statistics, manipulations, linalg and
estimators must keep their tensors on the GPU (native kernels where they exist) and still match
NumPy/SciPy and the reference fixtures. Checks that compare against host tensors by identity are
run with their device-independent parts only (see ``_HOST_ONLY``)."""
import importlib
import os

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "parity")
MODULES = sorted("tests.parity." + f[:-3] for f in os.listdir(HERE) if f.endswith("_checks.py"))
# host-by-construction checks (device switching, host-memory layout/sharing, printing of cpu:0)
_HOST_ONLY = {"core_misc::test_get_default_device_cpu", "core_misc::test_set_default_device_cpu",
              "core_misc::test_sanitize_device_cpu", "printing", "factories::test_asarray",
              "core_misc::test_sanitize_out"}
CASES = []
for _m in MODULES:
    _mod = importlib.import_module(_m)
    short = _m.rsplit(".", 1)[1].replace("_checks", "")
    for n in sorted(dir(_mod)):
        if n.startswith("test_") and callable(getattr(_mod, n)):
            if short in _HOST_ONLY or "{}::{}".format(short, n) in _HOST_ONLY:
                continue
            CASES.append((_m, n))


@pytest.mark.parametrize("module,name", CASES, ids=["{}::{}".format(m.rsplit(".", 1)[1][:-7], n) for m, n in CASES])
def test_parity_on_gpu(module, name, gpu):
    getattr(importlib.import_module(module), name)()
