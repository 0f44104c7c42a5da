"""Reference import path ``heat.core.tests.test_suites``."""
