"""The same checks in 2 and 3 gloo ranks (the reference runs its suite under mpirun -n 1..8)."""
import pytest

from . import dist_checks
from ._dist import run_distributed

CHECKS = [n for n in dir(dist_checks) if n.startswith("check_")]


@pytest.mark.parametrize("nprocs", [2, 3])
@pytest.mark.parametrize("name", CHECKS)
def test_distributed(name, nprocs):
    run_distributed("tests.dist_checks:" + name, nprocs)
