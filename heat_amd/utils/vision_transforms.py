"""Vision transforms (reference ``heat/utils/vision_transforms.py`` forwards to
``torchvision.transforms``; available when torchvision is installed)."""
try:
    import torchvision.transforms as _tvt
except ImportError:  # torchvision is optional
    _tvt = None


class TorchvisionMissing(AttributeError):
    """torchvision is not installed (an AttributeError, so ``getattr`` with a default and ``hasattr``
    keep working like for any missing attribute)."""


def __getattr__(name):
    if name.startswith("__"):
        raise AttributeError(name)
    if _tvt is None:
        raise TorchvisionMissing("torchvision is not installed; heat_amd.utils.vision_transforms.{} needs it"
                                 .format(name))
    try:
        return getattr(_tvt, name)
    except AttributeError:
        raise AttributeError("module {} has no attribute {}".format(__name__, name))
