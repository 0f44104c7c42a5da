"""Naive Bayes (reference ``heat/naive_bayes``)."""
from .gaussianNB import GaussianNB

__all__ = ["GaussianNB"]
