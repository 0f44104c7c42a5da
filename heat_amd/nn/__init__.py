"""Neural-network layers (reference ``heat/nn``): data-parallel wrappers plus every
``torch.nn`` name (module-level fall-through, like the reference)."""
import torch.nn as _tnn

from . import functional
from .data_parallel import DataParallel, DataParallelMultiGPU


def __getattr__(name):
    try:
        return getattr(_tnn, name)
    except AttributeError:
        raise AttributeError("module {} has no attribute {}".format(__name__, name))
