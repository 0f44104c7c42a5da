"""The scikit-learn / SciPy oracle checks (``tests/oracle_checks.py``) with the default device on
the MI355X (world of one): Lasso through the native Gram and sweep kernels, Lloyd through the
native assign/update kernels, distances through ``cdist_f16x3``/the exact kernel, moments and
percentiles through the fused moments and sort paths - all against the library implementations."""
import pytest

from . import oracle_checks

pytestmark = pytest.mark.gpu

CASES = [n for n in dir(oracle_checks) if n.startswith("check_")]


@pytest.mark.parametrize("name", CASES)
def test_oracle_on_gpu(name, gpu):
    getattr(oracle_checks, name)()
