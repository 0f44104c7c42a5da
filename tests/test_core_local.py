"""Every distributed check also runs in a world of one (in-process, CPU)."""
import pytest

from . import dist_checks

CHECKS = [n for n in dir(dist_checks) if n.startswith("check_")]


@pytest.mark.parametrize("name", CHECKS)
def test_local(name):
    getattr(dist_checks, name)()
