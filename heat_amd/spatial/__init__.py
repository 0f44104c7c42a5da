"""Spatial algorithms: pairwise distance / kernel matrices (reference ``heat/spatial``)."""
from .distance import *
