"""Mathematical constants (reference ``heat/core/constants.py``)."""
import math

__all__ = ["e", "Euler", "inf", "Inf", "Infty", "Infinity", "nan", "NaN", "pi"]

INF = math.inf
NAN = math.nan
NINF = -math.inf
PI = math.pi
E = math.e

inf = Inf = Infty = Infinity = INF
nan = NaN = NAN
pi = PI
e = Euler = E
