"""The multi-process checks with DEVICE buffers: 2 ranks share the one GPU of the test box
(RCCL refuses two ranks on one device, so the world group is gloo and every collective goes
through the host-staging wrappers of ``parallel/staging.py``). Every split-aware path the CPU
suite covers - Allreduce/Allgatherv/exchange/Bcast, ring passes, halos, native arg-reduce and
top-k, distributed Householder QR, k-means, cdist, moments - runs here on ``cuda:0`` tensors and
the native kernels, with the same NumPy oracles as ``test_distributed.py``."""
import pytest
import torch

from . import dist_checks, dist_checks_edge, dl_io_checks, oracle_checks, random_checks, vcoll_checks
from ._dist import run_distributed, run_distributed_batch

pytestmark = pytest.mark.gpu

MODULES = {"tests.dist_checks": dist_checks, "tests.dist_checks_edge": dist_checks_edge,
           "tests.random_checks": random_checks, "tests.oracle_checks": oracle_checks,
           "tests.dl_io_checks": dl_io_checks}
CASES = [(m, n) for m, mod in MODULES.items() for n in dir(mod) if n.startswith("check_")
         and getattr(getattr(mod, n), "__module__", m) == m]
ENV = {"HEAT_AMD_DEFAULT_DEVICE": "gpu", "HEAT_COMM_TIMEOUT": "60"}
_BATCH = {}


VCOLL = [n for n in dir(vcoll_checks) if n.startswith("check_")]


def _batch(module, nprocs=2, names=None):
    key = (module, nprocs)
    if key not in _BATCH:
        names = names or [n for m, n in CASES if m == module]
        _BATCH[key] = run_distributed_batch(module, names, nprocs, timeout=300, env_extra=ENV, keep_gpu=True)
    return _BATCH[key]


@pytest.mark.parametrize("module,name", CASES)
def test_distributed_on_device(module, name):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ok, err = _batch(module)[name]
    if not ok:
        pytest.fail("check {} failed with device buffers:\n{}".format(name, err))


CASES3 = [(m, n) for m, n in CASES if m in ("tests.dist_checks", "tests.dist_checks_edge")]


@pytest.mark.parametrize("module,name", CASES3)
def test_distributed_on_device_3_ranks(module, name):
    """The same checks at 3 ranks: every split of the check data is uneven (e.g. 40 rows -> 14 /
    13 / 13), so the offset / count / padding logic of the device paths runs off the even case."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ok, err = _batch(module, 3)[name]
    if not ok:
        pytest.fail("check {} failed with device buffers at 3 ranks:\n{}".format(name, err))


@pytest.mark.parametrize("nprocs", [3, 5])
@pytest.mark.parametrize("name", VCOLL)
def test_vcollectives_uneven_on_device(name, nprocs):
    """Allgatherv / Alltoallv / Gatherv / Scatterv / reduce-scatter with uneven and EMPTY blocks,
    device buffers, 3 and 5 ranks on the one card (``tests/vcoll_checks.py``)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ok, err = _batch("tests.vcoll_checks", nprocs, VCOLL)[name]
    if not ok:
        pytest.fail("check {} failed with device buffers at {} ranks:\n{}".format(name, nprocs, err))
