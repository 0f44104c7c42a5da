"""
The reference's data fixtures (``heat/datasets/iris.{csv,h5,nc}``, ``diabetes.h5``, the iris
train/test CSVs) and synthetic generators.

The fixture files are not shipped in this repository. :func:`fixture_path` finds them in
``$HEAT_DATASETS_DIR`` (e.g. a Heat checkout's ``heat/datasets``) or ``heat_amd/datasets/data``
and :func:`load_fixture` reads one in parallel through ``ht.load`` (CSV / HDF5 / NetCDF, split as
asked). :func:`iris` and :func:`diabetes` return the real fixture when one is found
(``synthetic=False``, the default) and otherwise a deterministic stand-in of the same shape and
character (3 Gaussian classes of 50 x 4 with the class means / spreads of Fisher's iris
measurements; a 442 x 11 linear-regression problem whose first column is the intercept, like the
fixture), identical on every rank for any process count.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from .. import core as ht
from ..core.dndarray import DNDarray

__all__ = ["iris", "diabetes", "make_blobs", "make_regression", "write_iris_csv", "fixture_path", "load_fixture",
           "FIXTURES"]

import os

# fixture file -> (dataset / variable name inside it or None for CSV, CSV separator)
FIXTURES = {
    "iris.csv": (None, ";"),
    "iris.h5": ("data", None),
    "iris.nc": ("data", None),
    "diabetes.h5": ("x", None),
    "iris_X_train.csv": (None, ";"),
    "iris_X_test.csv": (None, ";"),
    "iris_y_train.csv": (None, ";"),
    "iris_y_test.csv": (None, ";"),
    "iris_labels.csv": (None, ";"),
    "iris_y_pred_proba.csv": (None, ";"),
}


def _search_dirs():
    env = os.environ.get("HEAT_DATASETS_DIR")
    dirs = [env] if env else []
    dirs.append(os.path.join(os.path.dirname(os.path.abspath(__file__)), "data"))
    return dirs


def fixture_path(name: str) -> Optional[str]:
    """Path of the reference fixture ``name`` (e.g. ``"iris.h5"``) or None if none is found."""
    for d in _search_dirs():
        p = os.path.join(d, name)
        if os.path.isfile(p):
            return p
    return None


def load_fixture(name: str, dataset: Optional[str] = None, split: Optional[int] = 0, device=None, comm=None,
                 dtype=None) -> DNDarray:
    """Read the fixture ``name`` in parallel (``ht.load``: every rank reads its slab). ``dataset``
    overrides the dataset / variable of an HDF5 / NetCDF file (``diabetes.h5``: ``"x"`` or ``"y"``).
    Raises FileNotFoundError when the fixture is not available."""
    p = fixture_path(name)
    if p is None:
        raise FileNotFoundError("fixture {} not found in {}".format(name, _search_dirs()))
    ds, sep = FIXTURES.get(name, (None, ";"))
    kw = {"split": split, "device": device, "comm": comm}
    if dtype is not None:
        kw["dtype"] = dtype
    if p.endswith(".csv"):
        return ht.load(p, sep=sep, **kw)
    return ht.load(p, dataset if dataset is not None else ds, **kw)

_IRIS_MEANS = np.array([[5.006, 3.428, 1.462, 0.246], [5.936, 2.770, 4.260, 1.326], [6.588, 2.974, 5.552, 2.026]])
_IRIS_STDS = np.array([[0.352, 0.379, 0.174, 0.105], [0.516, 0.314, 0.470, 0.198], [0.636, 0.322, 0.552, 0.275]])


def _iris_numpy(seed: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    rng = np.random.default_rng(seed)
    X = np.concatenate([rng.normal(_IRIS_MEANS[c], _IRIS_STDS[c], size=(50, 4)) for c in range(3)])
    X = np.round(np.clip(X, 0.1, None), 1).astype(np.float32)
    y = np.repeat(np.arange(3), 50).astype(np.int64)
    return X, y


def iris(split: Optional[int] = 0, device=None, comm=None, seed: int = 0,
         synthetic: bool = False) -> Tuple[DNDarray, DNDarray]:
    """(150 x 4 float32 features, 150 int64 labels): Fisher's iris from the reference fixture
    (rows ordered by class, 50 each) when available, else the synthetic stand-in."""
    if not synthetic and fixture_path("iris.csv") is not None:
        X = load_fixture("iris.csv", split=split, device=device, comm=comm)
        y = np.repeat(np.arange(3), 50).astype(np.int64)
        return X, ht.array(y, split=split if split in (None, 0) else None, device=device, comm=comm)
    X, y = _iris_numpy(seed)
    return (ht.array(X, split=split, device=device, comm=comm),
            ht.array(y, split=split if split in (None, 0) else None, device=device, comm=comm))


def write_iris_csv(path: str, seed: int = 0, sep: str = ";") -> str:
    """Write the synthetic iris features as CSV (the reference loads ``iris.csv`` with ``sep=";"``)."""
    X, _ = _iris_numpy(seed)
    np.savetxt(path, X, delimiter=sep, fmt="%.1f")
    return path


def diabetes(split: Optional[int] = 0, device=None, comm=None, seed: int = 0,
             synthetic: bool = False) -> Tuple[DNDarray, DNDarray]:
    """442 x 11 features (first column = 1 for the Lasso intercept) and a (442, 1) target column:
    the reference's ``diabetes.h5`` (datasets ``x`` and ``y``) when available, else a synthetic
    problem of the same layout (442 x 11, column 0 the intercept)."""
    if not synthetic and fixture_path("diabetes.h5") is not None:
        X = load_fixture("diabetes.h5", "x", split=split, device=device, comm=comm)
        y = load_fixture("diabetes.h5", "y", split=split if split in (None, 0) else None, device=device, comm=comm)
        return X, ht.reshape(y, (-1, 1), new_split=y.split)
    X, y = make_regression(442, 10, noise=0.5, seed=seed, as_numpy=True)
    X = np.concatenate([np.ones((442, 1), np.float32), X], axis=1)
    return ht.array(X, split=split, device=device, comm=comm), ht.array(y, split=split, device=device, comm=comm)


def make_blobs(n_samples: int, centers: np.ndarray, std: float = 1.0, seed: int = 0, split: Optional[int] = 0,
               device=None, comm=None) -> Tuple[DNDarray, DNDarray]:
    """Isotropic Gaussian clusters around ``centers`` (k x f); balanced class sizes."""
    centers = np.asarray(centers, dtype=np.float64)
    k = centers.shape[0]
    rng = np.random.default_rng(seed)
    lab = np.arange(n_samples) % k
    X = (centers[lab] + std * rng.standard_normal((n_samples, centers.shape[1]))).astype(np.float32)
    return ht.array(X, split=split, device=device, comm=comm), ht.array(lab.astype(np.int64), split=split,
                                                                        device=device, comm=comm)


def make_regression(n_samples: int, n_features: int, noise: float = 0.1, sparsity: float = 0.5, seed: int = 0,
                    split: Optional[int] = 0, device=None, comm=None, as_numpy: bool = False):
    """y = X w + noise with unit mean-square columns and a sparse w (Lasso test problems)."""
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n_samples, n_features))
    X /= np.sqrt((X ** 2).mean(0))
    w = rng.standard_normal(n_features) * (rng.random(n_features) > sparsity)
    y = X @ w + noise * rng.standard_normal(n_samples)
    X, y = X.astype(np.float32), y.astype(np.float32)[:, None]
    if as_numpy:
        return X, y
    return ht.array(X, split=split, device=device, comm=comm), ht.array(y, split=split, device=device, comm=comm)
