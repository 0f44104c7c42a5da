"""Optimizers (reference ``heat/optim``): data-parallel wrappers plus every ``torch.optim`` name."""
import torch.optim as _topt

from . import lr_scheduler, utils
from .dp_optimizer import DASO, DataParallelOptimizer
from .utils import DetectMetricPlateau


def __getattr__(name):
    try:
        return getattr(_topt, name)
    except AttributeError:
        raise AttributeError("module {} has no attribute {}".format(__name__, name))
