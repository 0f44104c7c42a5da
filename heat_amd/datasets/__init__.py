"""
Synthetic stand-ins for the reference's data fixtures (``heat/datasets/iris.{csv,h5,nc}``,
``diabetes.h5``). The files themselves are not shipped: these generators produce
deterministic data of the same shape and character (3 Gaussian classes of 50 x 4 with the class
means/spreads of Fisher's iris measurements; a 442 x 10 linear-regression problem), identical on
every rank and for any process count, returned as split DNDarrays.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from .. import core as ht
from ..core.dndarray import DNDarray

__all__ = ["iris", "diabetes", "make_blobs", "make_regression", "write_iris_csv"]

_IRIS_MEANS = np.array([[5.006, 3.428, 1.462, 0.246], [5.936, 2.770, 4.260, 1.326], [6.588, 2.974, 5.552, 2.026]])
_IRIS_STDS = np.array([[0.352, 0.379, 0.174, 0.105], [0.516, 0.314, 0.470, 0.198], [0.636, 0.322, 0.552, 0.275]])


def _iris_numpy(seed: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    rng = np.random.default_rng(seed)
    X = np.concatenate([rng.normal(_IRIS_MEANS[c], _IRIS_STDS[c], size=(50, 4)) for c in range(3)])
    X = np.round(np.clip(X, 0.1, None), 1).astype(np.float32)
    y = np.repeat(np.arange(3), 50).astype(np.int64)
    return X, y


def iris(split: Optional[int] = 0, device=None, comm=None, seed: int = 0) -> Tuple[DNDarray, DNDarray]:
    """(150 x 4 float32 features, 150 int64 labels) with iris-like class structure."""
    X, y = _iris_numpy(seed)
    return (ht.array(X, split=split, device=device, comm=comm),
            ht.array(y, split=split if split in (None, 0) else None, device=device, comm=comm))


def write_iris_csv(path: str, seed: int = 0, sep: str = ";") -> str:
    """Write the synthetic iris features as CSV (the reference loads ``iris.csv`` with ``sep=";"``)."""
    X, _ = _iris_numpy(seed)
    np.savetxt(path, X, delimiter=sep, fmt="%.1f")
    return path


def diabetes(split: Optional[int] = 0, device=None, comm=None, seed: int = 0) -> Tuple[DNDarray, DNDarray]:
    """442 x 10 standardised features (first column = 1 for the Lasso intercept) and targets."""
    X, y = make_regression(442, 10, noise=0.5, seed=seed, as_numpy=True)
    X[:, 0] = 1.0
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
