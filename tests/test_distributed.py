"""The same checks in 2, 3, 4, 5 and 8 gloo ranks (the reference runs its whole suite under
``mpirun -n 1..8``, Jenkinsfile:19-26; the world of one runs in ``test_core_local.py``).

All checks of one (module, world size) run in ONE multi-rank job (interpreter start-up dominated
the per-check runs); a failing check is re-run alone in a fresh job to report a clean traceback."""
import pytest

from . import dist_checks, dist_checks_edge, dl_io_checks, oracle_checks, random_checks, vcoll_checks
from ._dist import run_distributed, run_distributed_batch

MODULES = {"tests.dist_checks": dist_checks, "tests.dist_checks_edge": dist_checks_edge,
           "tests.vcoll_checks": vcoll_checks, "tests.random_checks": random_checks,
           "tests.oracle_checks": oracle_checks, "tests.dl_io_checks": dl_io_checks}
CASES = [(m, n) for m, mod in MODULES.items() for n in dir(mod) if n.startswith("check_")
         and getattr(getattr(mod, n), "__module__", m) == m]
_BATCH = {}


def _batch(module, nprocs, staged=False):
    key = (module, nprocs, staged)
    if key not in _BATCH:
        names = [n for m, n in CASES if m == module]
        env = {"HEAT_COMM_FORCE_STAGING": "1"} if staged else None
        _BATCH[key] = run_distributed_batch(module, names, nprocs, env_extra=env)
    return _BATCH[key]


@pytest.mark.parametrize("nprocs", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("module,name", CASES)
def test_distributed(module, name, nprocs):
    ok, err = _batch(module, nprocs)[name]
    if not ok:
        run_distributed(module + ":" + name, nprocs)  # raises with the full per-rank log
        pytest.fail("check {} failed in the batched job but passed alone:\n{}".format(name, err))


@pytest.mark.parametrize("module,name", CASES)
def test_distributed_host_staged(module, name):
    """Every collective through the host-staging wrappers (``parallel/staging.py``: copy out,
    gloo, copy back on ``wait()``), the path device buffers take on a gloo-only group."""
    ok, err = _batch(module, 3, staged=True)[name]
    if not ok:
        run_distributed(module + ":" + name, 3, env_extra={"HEAT_COMM_FORCE_STAGING": "1"})
        pytest.fail("check {} failed in the batched job but passed alone:\n{}".format(name, err))
