"""Functional interface: every ``torch.nn.functional`` name (reference ``heat/nn/functional.py``)."""
import torch.nn.functional as _F


def __getattr__(name):
    try:
        return getattr(_F, name)
    except AttributeError:
        raise AttributeError("module {} has no attribute {}".format(__name__, name))
