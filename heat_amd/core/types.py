"""
Heat-compatible scalar type system.

Behavioural parity with the reference's ``heat/core/types.py`` (class hierarchy 64-412, aliases
415-428, ``canonical_heat_type`` 495, ``heat_type_of`` 565, cast tables 619-666, ``can_cast`` 671,
promotion table 755, ``result_type`` 868, ``finfo/iinfo`` 950/1007).

The promotion table is not hard-coded: it is derived from the "intuitive" cast relation (the
smallest type both operands can be intuitively cast to), exactly like the reference defines it.
The tables themselves are generated from a small set of rules instead of being spelled out.
"""
from __future__ import annotations

import builtins
from typing import Any, Type, Union

import numpy as np
import torch

__all__ = [
    "datatype", "number", "integer", "signedinteger", "unsignedinteger", "bool", "bool_",
    "floating", "int8", "byte", "int16", "short", "int32", "int", "int64", "long", "uint8",
    "ubyte", "float32", "float", "float_", "float64", "double", "flexible", "can_cast",
    "canonical_heat_type", "heat_type_is_exact", "heat_type_is_inexact", "heat_type_is_complexfloating",
    "iscomplex", "isreal", "issubdtype", "heat_type_of", "promote_types", "result_type",
    "complex64", "cfloat", "csingle", "complex128", "cdouble", "finfo", "iinfo", "complex",
]


class datatype:
    """Base of all heat types. Calling a type casts its arguments into a DNDarray of that type."""

    _torch = None
    _char = None

    def __new__(cls, *value, device=None, comm=None):
        from . import factories

        torch_type = cls.torch_type()
        if torch_type is None:
            raise TypeError("cannot create '{}' instances".format(cls))
        n = len(value)
        if n == 0:
            value = ((0,),)
        if len(value) > 1:
            raise TypeError("{} takes at most one positional argument, got {}".format(cls.__name__, n))
        value = value[0]
        from .dndarray import DNDarray

        if isinstance(value, DNDarray):
            return value.astype(cls)
        return factories.array(value, dtype=cls, device=device, comm=comm)

    @classmethod
    def torch_type(cls):
        return cls._torch

    @classmethod
    def char(cls):
        """The type's array-protocol code like the reference ('i4', 'f4', 'c8', bool: 'u1')."""
        return _TYPESTR.get(cls, cls._char)


class bool(datatype):
    _torch = torch.bool
    _char = "?"


class number(datatype):
    pass


class integer(number):
    pass


class signedinteger(integer):
    pass


class int8(signedinteger):
    _torch = torch.int8
    _char = "b"


class int16(signedinteger):
    _torch = torch.int16
    _char = "h"


class int32(signedinteger):
    _torch = torch.int32
    _char = "i"


class int64(signedinteger):
    _torch = torch.int64
    _char = "l"


class unsignedinteger(integer):
    pass


class uint8(unsignedinteger):
    _torch = torch.uint8
    _char = "B"


class floating(number):
    pass


class float32(floating):
    _torch = torch.float32
    _char = "f"


class float64(floating):
    _torch = torch.float64
    _char = "d"


class complex(number):
    pass


class complex64(complex):
    _torch = torch.complex64
    _char = "F"


class complex128(complex):
    _torch = torch.complex128
    _char = "D"


class flexible(datatype):
    pass


# aliases (reference types.py:415-428)
bool_ = bool
ubyte = uint8
byte = int8
short = int16
int = int32
int_ = int32
long = int64
float = float32
float_ = float32
double = float64
cfloat = complex64
csingle = complex64
cdouble = complex128

_complexfloating = (complex64, complex128)
_inexact = (float32, float64, complex64, complex128)
_exact = (uint8, int8, int16, int32, int64)

# ordering used by the cast tables: the index is the "type code"
_ORDER = (bool, uint8, int8, int16, int32, int64, float32, float64, complex64, complex128)
_CODE = {t: i for i, t in enumerate(_ORDER)}

_by_char = {t._char: t for t in _ORDER}
_TYPESTR = {bool: "u1", uint8: "u1", int8: "i1", int16: "i2", int32: "i4", int64: "i8", float32: "f4",
            float64: "f8", complex64: "c8", complex128: "c16"}
_by_str = {
    "b1": bool, "u": uint8, "u1": uint8, "i1": int8, "i2": int16, "i4": int32, "i8": int64,
    "f4": float32, "f8": float64, "c8": complex64, "c16": complex128,
    "bool": bool, "uint8": uint8, "int8": int8, "int16": int16, "int32": int32, "int64": int64,
    "float32": float32, "float64": float64, "complex64": complex64, "complex128": complex128,
}
_by_torch = {t._torch: t for t in _ORDER}
_by_numpy = {np.dtype(t._char).type: t for t in _ORDER}
_by_builtin = {builtins.bool: bool, builtins.int: int32, builtins.float: float32,
               builtins.complex: complex64}


def canonical_heat_type(a_type: Union[str, Type[datatype], Any]) -> Type[datatype]:
    """Canonicalise a builtin/numpy/torch type, a type string or a heat type into a heat type."""
    if isinstance(a_type, type) and issubclass(a_type, datatype):
        if a_type._torch is None:
            raise TypeError("data type {} is abstract".format(a_type))
        return a_type
    try:
        if isinstance(a_type, str):
            if a_type in _by_char:
                return _by_char[a_type]
            return _by_str[a_type]
        if isinstance(a_type, torch.dtype):
            return _by_torch[a_type]
        if isinstance(a_type, np.dtype):
            return _by_numpy[a_type.type]
        if a_type in _by_builtin:
            return _by_builtin[a_type]
        if a_type in _by_numpy:
            return _by_numpy[a_type]
    except (KeyError, TypeError):
        pass
    raise TypeError("data type {} is not understood".format(a_type))


def heat_type_of(obj) -> Type[datatype]:
    """Infer the heat type of an object (array, tensor, scalar, sequence)."""
    from .dndarray import DNDarray

    if isinstance(obj, DNDarray):
        return obj.dtype
    if isinstance(obj, torch.Tensor):
        return canonical_heat_type(obj.dtype)
    if isinstance(obj, np.ndarray):
        return canonical_heat_type(obj.dtype)
    if isinstance(obj, (np.generic,)):
        return canonical_heat_type(obj.dtype)
    if isinstance(obj, (builtins.bool, builtins.int, builtins.float, builtins.complex)):
        return canonical_heat_type(type(obj))
    if isinstance(obj, (list, tuple)):
        try:
            return canonical_heat_type(np.asarray(obj).dtype)
        except Exception:
            # mixed sequences: the type of the first element, like the reference
            if len(obj):
                return heat_type_of(obj[0])
    if isinstance(obj, type):
        return canonical_heat_type(obj)
    raise TypeError("data type of {} is not understood".format(obj))


def heat_type_is_exact(ht_dtype) -> builtins.bool:
    """True for the exact (boolean and integer) heat types."""
    return canonical_heat_type(ht_dtype) in _exact


def heat_type_is_inexact(ht_dtype) -> builtins.bool:
    """True for the floating-point and complex heat types."""
    return canonical_heat_type(ht_dtype) in _inexact


def heat_type_is_complexfloating(ht_dtype) -> builtins.bool:
    """True for complex64 / complex128."""
    return canonical_heat_type(ht_dtype) in _complexfloating


def _kind(t) -> builtins.int:
    # 0 bool, 1 unsigned, 2 signed, 3 float, 4 complex
    if t is bool:
        return 0
    if t is uint8:
        return 1
    if issubclass(t, signedinteger):
        return 2
    if issubclass(t, floating):
        return 3
    return 4


def _bits(t) -> builtins.int:
    return {bool: 1, uint8: 8, int8: 8, int16: 16, int32: 32, int64: 64, float32: 32,
            float64: 64, complex64: 64, complex128: 128}[t]


def _mantissa(t) -> builtins.int:
    # significand bits of the real component (exactly representable integer range)
    return {float32: 24, float64: 53, complex64: 24, complex128: 53}[t]


def _safe(a, b) -> builtins.bool:
    """numpy "safe" casting among the ten heat types."""
    if a is b or a is bool:
        return True
    ka, kb = _kind(a), _kind(b)
    if kb == 0:
        return False
    if ka in (1, 2) and kb in (1, 2):
        if ka == kb:
            return _bits(b) >= _bits(a)
        if ka == 1:  # unsigned -> signed needs one more bit
            return _bits(b) > _bits(a)
        return False  # signed -> unsigned never safe
    if ka in (1, 2) and kb >= 3:
        # 8/16-bit integers fit any float; wider ones need a 53-bit significand
        return _bits(a) <= 16 or _mantissa(b) == 53
    if ka == 3 and kb == 3:
        return _bits(b) >= _bits(a)
    if ka == 3 and kb == 4:
        return _mantissa(b) >= _mantissa(a)
    if ka == 4 and kb == 4:
        return _bits(b) >= _bits(a)
    return False


def _intuitive(a, b) -> builtins.bool:
    """safe casting plus int32 -> float32 / complex64 (same bit width), reference types.py:639-651."""
    if _safe(a, b):
        return True
    return a is int32 and b in (float32, complex64)


def _same_kind(a, b) -> builtins.bool:
    ka, kb = _kind(a), _kind(b)
    if ka in (1, 2) and kb in (1, 2):
        return True
    return ka == kb or _safe(a, b)


_CAST_KINDS = ("no", "safe", "same_kind", "unsafe", "intuitive")


def can_cast(from_, to, casting: str = "intuitive") -> builtins.bool:
    """Whether a cast is possible under the given rule; scalars are checked by value."""
    if not isinstance(casting, str):
        raise TypeError("expected string, found {}".format(type(casting)))
    if casting not in _CAST_KINDS:
        raise ValueError("casting must be one of {}".format(str(_CAST_KINDS)[1:-1]))
    to_t = canonical_heat_type(to)
    try:
        from_t = canonical_heat_type(from_)
    except TypeError:
        from_t = heat_type_of(from_)
        # scalar value check (numpy semantics: value fits)
        if casting not in ("unsafe", "no") and isinstance(from_, (builtins.int, builtins.float)) \
                and not isinstance(from_, builtins.bool):
            if heat_type_is_exact(to_t) and isinstance(from_, builtins.int):
                info = torch.iinfo(to_t._torch)
                return info.min <= from_ <= info.max
            if heat_type_is_exact(to_t) and isinstance(from_, builtins.float):
                return False
            if to_t in (float32, complex64):
                return abs(from_) <= torch.finfo(torch.float32).max or from_ != from_
            return True
    if casting == "unsafe":
        return True
    if casting == "no":
        return from_t is to_t
    if casting == "safe":
        return _safe(from_t, to_t)
    if casting == "intuitive":
        return _intuitive(from_t, to_t)
    return _same_kind(from_t, to_t)


# promotion table derived from the intuitive cast relation (reference types.py:755-761)
_PROMOTE = [[None] * len(_ORDER) for _ in _ORDER]
for _i, _a in enumerate(_ORDER):
    for _j, _b in enumerate(_ORDER):
        for _t in _ORDER:
            if _intuitive(_a, _t) and _intuitive(_b, _t):
                _PROMOTE[_i][_j] = _t
                break


def promote_types(type1, type2) -> Type[datatype]:
    """Smallest type both operands can be intuitively cast to (symmetric)."""
    return _PROMOTE[_CODE[canonical_heat_type(type1)]][_CODE[canonical_heat_type(type2)]]


def issubdtype(arg1, arg2) -> builtins.bool:
    """numpy-style ``issubdtype``: whether ``arg1`` is ``arg2`` or below it in the heat type hierarchy
    (arguments may be heat types, torch / numpy dtypes or their names)."""
    if not (isinstance(arg1, type) and issubclass(arg1, datatype)):
        arg1 = canonical_heat_type(arg1)
    if not (isinstance(arg2, type) and issubclass(arg2, datatype)):
        arg2 = canonical_heat_type(arg2)
    return issubclass(arg1, arg2)


def _type_and_precedence(arg):
    """precedence: 0 array, 1 type, 2 0-d array, 3 python scalar (lower wins)."""
    from .dndarray import DNDarray

    if isinstance(arg, (DNDarray, torch.Tensor, np.ndarray)):
        t = heat_type_of(arg)
        return t, (0 if len(arg.shape) > 0 else 2)
    if isinstance(arg, np.generic):
        return canonical_heat_type(arg.dtype), 2
    try:
        if isinstance(arg, np.dtype):
            arg = arg.char
        return canonical_heat_type(arg), 1
    except TypeError:
        return canonical_heat_type(type(arg)), 3


def result_type(*arrays_and_types) -> Type[datatype]:
    """Type resulting from an arithmetic operation of the given operands (reference types.py:868)."""
    t, p = _type_and_precedence(arrays_and_types[-1])
    for arg in reversed(arrays_and_types[:-1]):
        t1, p1 = _type_and_precedence(arg)
        if t1 is t:
            p = min(p, p1)
            continue
        if p1 == p:
            t = promote_types(t1, t)
            continue
        same = None
        for sclass in (bool, integer, floating, complex):
            if issubclass(t1, sclass) and issubclass(t, sclass):
                same = sclass
                break
        if same is not None:
            t = t1 if p1 < p else t
        else:
            t = t if _CODE[t1] < _CODE[t] else t1
        p = min(p, p1)
    return t


def iscomplex(x):
    """Element-wise: True where the imaginary part is non-zero (all False for a real dtype)."""
    from . import factories, _operations

    if issubclass(x.dtype, _complexfloating):
        return x.imag != 0
    return factories.zeros(x.shape, bool, split=x.split, device=x.device, comm=x.comm)


def isreal(x):
    """Element-wise: True where the imaginary part is zero (all True for a real dtype)."""
    from . import _operations

    return _operations.local_op(torch.isreal, x, no_cast=True)


class finfo:
    """Machine limits of floating point heat types."""

    def __new__(cls, dtype):
        try:
            dtype = heat_type_of(dtype)
        except (KeyError, IndexError, TypeError):
            pass
        if dtype not in _inexact:
            raise TypeError("Data type {} not inexact, not supported".format(dtype))
        self = super().__new__(cls)
        info = torch.finfo(dtype._torch)
        self.bits, self.eps, self.max, self.tiny = info.bits, info.eps, info.max, info.tiny
        self.min = -self.max
        return self


class iinfo:
    """Machine limits of integer heat types."""

    def __new__(cls, dtype):
        try:
            dtype = heat_type_of(dtype)
        except (KeyError, IndexError, TypeError):
            pass
        if dtype not in _exact:
            raise TypeError("Data type {} not exact, not supported".format(dtype))
        self = super().__new__(cls)
        info = torch.iinfo(dtype._torch)
        self.bits, self.max = info.bits, info.max
        self.min = -(self.max + 1)
        return self
