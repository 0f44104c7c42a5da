"""Classification (reference ``heat/classification``)."""
from .kneighborsclassifier import KNeighborsClassifier

__all__ = ["KNeighborsClassifier"]
