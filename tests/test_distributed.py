"""The same checks in 2 and 3 gloo ranks (the reference runs its suite under mpirun -n 1..8).

All checks of one world size run in ONE multi-rank job (interpreter start-up dominated the
per-check runs); a failing check is re-run alone in a fresh job to report a clean traceback."""
import pytest

from . import dist_checks
from ._dist import run_distributed, run_distributed_batch

CHECKS = [n for n in dir(dist_checks) if n.startswith("check_")]
_BATCH = {}


def _batch(nprocs):
    if nprocs not in _BATCH:
        _BATCH[nprocs] = run_distributed_batch("tests.dist_checks", CHECKS, nprocs)
    return _BATCH[nprocs]


@pytest.mark.parametrize("nprocs", [2, 3])
@pytest.mark.parametrize("name", CHECKS)
def test_distributed(name, nprocs):
    ok, err = _batch(nprocs)[name]
    if not ok:
        run_distributed("tests.dist_checks:" + name, nprocs)  # raises with the full per-rank log
        pytest.fail("check {} failed in the batched job but passed alone:\n{}".format(name, err))
