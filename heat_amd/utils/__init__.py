"""Utilities (reference ``heat/utils``): data loading helpers and vision transforms."""
from . import data
from . import vision_transforms
