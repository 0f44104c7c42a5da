"""Every distributed check also runs in a world of one (in-process, CPU)."""
import pytest

from . import dist_checks, dist_checks_edge, oracle_checks, random_checks

CASES = [(mod, n) for mod in (dist_checks, dist_checks_edge, random_checks, oracle_checks) for n in dir(mod)
         if n.startswith("check_") and getattr(mod, n).__module__ == mod.__name__]


@pytest.mark.parametrize("mod,name", CASES, ids=[n for _, n in CASES])
def test_local(mod, name):
    getattr(mod, name)()
