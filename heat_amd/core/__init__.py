"""Core of the framework: the distributed array, its type system and the NumPy-like op library
(reference ``heat/core/__init__.py``)."""
from .constants import *
from .arithmetics import *
from .base import *
from .communication import *
from .complex_math import *
from .constants import *
from .devices import *
from .exponential import *
from .dndarray import *
from .factories import *
from .indexing import *
from .io import *
from .linalg import *
from .logical import *
from .manipulations import *
from .memory import *
from .printing import *
from . import random
from .relational import *
from .rounding import *
from .sanitation import *
from .statistics import *
from .stride_tricks import *
from .tiling import *
from .trigonometrics import *
from .types import *
from .types import finfo, iinfo
from . import version
from .version import __version__
from .io import load, save
