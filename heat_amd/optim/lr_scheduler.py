"""Learning-rate schedulers: every ``torch.optim.lr_scheduler`` name is available here
(reference ``heat/optim/lr_scheduler.py`` falls through to torch the same way)."""
import torch.optim.lr_scheduler as _tls


def __getattr__(name):
    try:
        return getattr(_tls, name)
    except AttributeError:
        raise AttributeError("module {} has no attribute {}".format(__name__, name))
