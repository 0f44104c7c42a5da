"""Reference import path ``heat.core.tests.test_suites.basic_test`` for downstream test suites; the
implementation is :mod:`heat_amd.testing`."""
from ....testing import TestCase  # noqa: F401
