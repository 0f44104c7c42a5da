"""Regression estimators (reference ``heat/regression``)."""
from .lasso import *
