"""Vision transforms (reference ``heat/utils/vision_transforms.py`` forwards to
``torchvision.transforms``; available when torchvision is installed)."""
try:
    import torchvision.transforms as _tvt
except ImportError:  # torchvision is optional
    _tvt = None


def __getattr__(name):
    if _tvt is None:
        raise ImportError("torchvision is not installed; heat_amd.utils.vision_transforms needs it")
    try:
        return getattr(_tvt, name)
    except AttributeError:
        raise AttributeError("module {} has no attribute {}".format(__name__, name))
