"""Functional interface: every ``torch.nn.functional`` name (reference ``heat/nn/functional.py``)."""
import torch.nn.functional as _F


def func_getattr(name):
    """Resolve ``name`` in ``torch.nn.functional`` (module-level fall-through)."""
    try:
        return getattr(_F, name)
    except AttributeError:
        raise AttributeError("module {} has no attribute {}".format(__name__, name))


__getattr__ = func_getattr
