"""
Lasso regression by cyclic coordinate descent (reference ``heat/regression/lasso.py``: ``Lasso`` 10,
``soft_threshold`` 90, ``rmse`` 108, ``fit`` 121-175, ``predict`` 177).

Same objective, same update rule (feature 0 is the intercept column and is not thresholded), but
O(m n) per sweep instead of O(m n^2): the residual stays on the device and every coordinate is
one fused native pass (``ops.lasso_epoch``) plus, for split data, one scalar all-reduce.

Narrow problems (n <= 64 features, the tall-skinny regime the reference benchmarks) take the
covariance form of the same update: rho_j = b_j - (G theta)_j + G_jj theta_j with G = X^T X / m,
b = X^T y / m. One native pass over the rows builds [X | y]^T [X | y] (``ops.lasso_gram``), split
data needs ONE fp64 all-reduce of that (n+1)^2 matrix per fit, and every sweep plus the convergence
test runs in one single-wavefront kernel (``ops.lasso_cd``). Wider device problems (n <= 2048)
take the same form when a measured cost model (``_prefer_gram``) says the Gram GEMM is cheaper than
max_iter data sweeps. ``HEAT_LASSO_SOLVER=sweep|gram`` forces either form.
"""
from __future__ import annotations

import os
from typing import Optional, Union

import torch

from .. import core as ht
from ..core.base import BaseEstimator, RegressionMixin
from ..core.communication import MPI
from ..core.dndarray import DNDarray
from .. import ops

__all__ = ["Lasso"]


def _prefer_gram(m_local: int, n: int, max_iter: int, device: bool) -> bool:
    """Covariance vs sweep solver by a cost model with constants measured on one MI355X (1e7 rows,
    n = 16 / 256: a sweep costs ~60 us per coordinate, one column pass at ~0.7 TB/s; the Gram pass
    runs at ~4 TB/s (native, n < 24) or as a batched fp32 GEMM at ~130 TFLOP/s; device CD ~0.1 us
    per coordinate plus n/64 L2 loads)."""
    if n <= 64:
        return True
    if not device or n > 2048:
        return False
    sweep = max_iter * n * (4.0 * m_local / 0.7e12 + 3e-6)
    gram = 2.0 * m_local * n * n / 1.3e14 + 4.0 * m_local * n / 4e12 + max_iter * n * (1e-7 + n / 64 * 2e-9)
    return gram < sweep


class Lasso(RegressionMixin, BaseEstimator):
    """Least absolute shrinkage and selection operator: min 1/(2m)|y - Xw|^2 + lam |w_1:|_1."""

    def __init__(self, lam: Optional[float] = 0.1, max_iter: Optional[int] = 100, tol: Optional[float] = 1e-6) -> None:
        self.__lam = lam
        self.max_iter = max_iter
        self.tol = tol
        self.__theta = None
        self.n_iter = None

    @property
    def coef_(self) -> Optional[DNDarray]:
        return None if self.__theta is None else self.__theta[1:]

    @property
    def intercept_(self) -> Optional[DNDarray]:
        return None if self.__theta is None else self.__theta[0]

    @property
    def lam(self) -> float:
        return self.__lam

    @lam.setter
    def lam(self, arg: float) -> None:
        self.__lam = arg

    @property
    def theta(self) -> Optional[DNDarray]:
        return self.__theta

    def soft_threshold(self, rho):
        """Soft-threshold operator ``S(rho, lam)``."""
        lam = self.__lam
        if isinstance(rho, DNDarray):
            rho = rho.item()
        if rho < -lam:
            return rho + lam
        if rho > lam:
            return rho - lam
        return 0.0

    def rmse(self, gt: DNDarray, yest: DNDarray) -> float:
        """Root mean square error between two arrays."""
        return float(ht.sqrt(ht.mean((gt - yest) ** 2)).item())

    def fit(self, x: DNDarray, y: DNDarray) -> None:
        """Coordinate descent until the RMS change of theta is below ``tol`` or ``max_iter`` sweeps."""
        if y.ndim > 2:
            raise ValueError("y.ndim must <= 2, currently: {}".format(y.ndim))
        if x.ndim != 2:
            raise ValueError("X.ndim must == 2, currently: {}".format(x.ndim))
        if x.split not in (None, 0):
            raise NotImplementedError("Lasso supports split=None or split=0 inputs")
        m, n = x.gshape
        X = x.larray
        if not X.is_floating_point():
            X = X.float()
        tt = X.dtype if X.dtype in (torch.float32, torch.float64) else torch.float32
        X = X.to(tt)
        if y.gnumel != m:
            raise ValueError("y must hold one target per row of x: {} != {}".format(y.gnumel, m))
        # y's local rows must be exactly x's local rows (the native kernels index both by row)
        if y.ndim != 1:
            # (m, 1) / (1, m) targets of any split -> 1-D (split 0 if distributed, C order)
            y = ht.reshape(y, (m,), new_split=0 if y.split is not None else None)
        if x.is_distributed():
            if y.split is None:
                counts, displs = x.counts_displs()
                r0 = displs[x.comm.rank]
                yl = y.larray.reshape(-1)[r0: r0 + counts[x.comm.rank]]
            else:
                yl = y.larray if y.split_counts() == x.split_counts() else \
                    y._exchange_rows(y.split_counts(), x.split_counts())
                yl = yl.reshape(-1)
        else:
            yl = (ht.resplit(y, None) if y.is_distributed() else y).larray.reshape(-1)
        yl = yl.to(device=X.device, dtype=tt)
        if yl.numel() != X.shape[0]:
            raise ValueError("local rows of x ({}) and y ({}) differ".format(X.shape[0], yl.numel()))
        dist = x.is_distributed()
        solver = os.environ.get("HEAT_LASSO_SOLVER", "auto")
        # the cost model sees the rows this rank really processes (all m when x is replicated)
        if solver == "gram" or (solver == "auto" and _prefer_gram(X.shape[0], n, self.max_iter, X.is_cuda)):
            G = ops.lasso_gram(X, yl)                         # [n+1, n+1] fp64, local rows
            if dist:
                x.comm.Allreduce(MPI.IN_PLACE, G, MPI.SUM)
            G = G / m
            th = torch.zeros(n, dtype=torch.float64, device=X.device)
            it = ops.lasso_cd(G[:n, :n], G[:n, n].contiguous(), float(self.__lam), int(self.max_iter), self.tol, th)
            self.n_iter = it
            self.__theta = DNDarray(th.to(tt).reshape(n, 1), (n, 1), ht.types.canonical_heat_type(tt), None, x.device,
                                    x.comm, True)
            return
        XT, colsq = ops.lasso_prepare(X)                       # [n, m_local]: features contiguous
        if dist:
            x.comm.Allreduce(MPI.IN_PLACE, colsq, MPI.SUM)
        colsq = colsq / m
        theta = torch.zeros(n, dtype=tt, device=X.device)
        r = yl.clone()                                        # residual y - X theta (theta = 0)

        def allreduce(t):
            x.comm.Allreduce(MPI.IN_PLACE, t, MPI.SUM)

        i = 0
        sweep = ops.LassoSweep(XT, r, theta, colsq, float(self.__lam), m, allreduce if dist else None,
                               use_graph=self.max_iter >= 3)  # capture pays off from the 3rd sweep
        for i in range(self.max_iter):
            theta_old = theta.clone()
            sweep()
            if self.tol is not None:
                diff = float(torch.sqrt(torch.mean((theta - theta_old) ** 2)))
                if diff < self.tol:
                    break
        self.n_iter = i + 1
        self.__theta = DNDarray(theta.reshape(n, 1), (n, 1), ht.types.canonical_heat_type(tt), None, x.device, x.comm,
                                True)

    def predict(self, x: DNDarray) -> DNDarray:
        """``x @ theta`` (the first column of x multiplies the intercept)."""
        return ht.matmul(x, self.__theta.astype(x.dtype) if x.dtype != self.__theta.dtype else self.__theta)
