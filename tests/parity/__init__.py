"""Reference-parity checks: one module per reference test file (``heat/*/tests/test_<name>.py``)
with a check of the same name for every reference test method, written against NumPy / PyTorch
oracles. ``tests/test_parity.py`` runs each in a world of one and in 2, 3, 5 and 8 gloo ranks."""
