"""Optimizers (reference ``heat/optim``)."""
