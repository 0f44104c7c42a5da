"""Distributed data loading (reference ``heat/utils/data``)."""
from .datatools import *
from .partial_dataset import *
from .mnist import *
from . import matrixgallery
