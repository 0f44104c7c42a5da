"""Reference import path ``heat.core.tests`` (the test base class lives in :mod:`heat_amd.testing`)."""
