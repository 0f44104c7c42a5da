"""
Gaussian Naive Bayes (reference ``heat/naive_bayes/gaussianNB.py``: ``GaussianNB`` 12, ``fit`` 70,
``partial_fit`` 200, ``__update_mean_variance`` 131 (Chan et al. merge), ``__joint_log_likelihood``
391, ``logsumexp`` 407, ``predict(_log)_proba`` 480-529).

All classes are updated together: one segmented pass (per-class weighted count / sum / squared
deviation via ``index_add``) and ONE all-reduce of the packed per-class moments, then the Chan
merge with the previous state (the reference loops over classes with a distributed mean/var each).
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch

from .. import core as ht
from ..core.base import BaseEstimator, ClassificationMixin
from ..core.communication import MPI
from ..core.dndarray import DNDarray

__all__ = ["GaussianNB"]


class GaussianNB(ClassificationMixin, BaseEstimator):
    """Gaussian Naive Bayes with online updates (``partial_fit``)."""

    @property
    def epsilon_(self) -> DNDarray:
        """Variance floor added to every class variance: var_smoothing * max feature variance
        (shape (1,), like the reference); an AttributeError before the first fit."""
        if getattr(self, "_epsilon", None) is None:
            raise AttributeError("'GaussianNB' object has no attribute 'epsilon_' (not fitted yet)")
        return ht.array([self._epsilon], dtype=ht.float64)

    def __init__(self, priors=None, var_smoothing: float = 1e-9):
        self.priors = priors
        self.var_smoothing = var_smoothing

    # ----------------------------------------------------------------- fitting
    def fit(self, x: DNDarray, y: DNDarray, sample_weight: Optional[DNDarray] = None) -> "GaussianNB":
        if not isinstance(x, DNDarray):
            raise ValueError("input needs to be a ht.DNDarray, but was {}".format(type(x)))
        if not isinstance(y, DNDarray):
            raise ValueError("input needs to be a ht.DNDarray, but was {}".format(type(y)))
        if y.ndim != 1:
            raise ValueError("expected y to be a 1-D tensor, is {}-D".format(y.ndim))
        if sample_weight is not None and not isinstance(sample_weight, DNDarray):
            raise ValueError("sample_weight needs to be a ht.DNDarray, but was {}".format(type(sample_weight)))
        classes = ht.unique(y, sorted=True)
        if classes.split is not None:
            classes = ht.resplit(classes, None)
        return self._partial_fit(x, y, classes, _refit=True, sample_weight=sample_weight)

    def partial_fit(self, x: DNDarray, y: DNDarray, classes: Optional[DNDarray] = None,
                    sample_weight: Optional[DNDarray] = None) -> "GaussianNB":
        return self._partial_fit(x, y, classes, _refit=False, sample_weight=sample_weight)

    def _local_rows(self, arr: DNDarray, like: DNDarray) -> torch.Tensor:
        """``arr``'s rows aligned with ``like``'s local rows."""
        if arr.split == like.split and arr.split_counts() == like.split_counts():
            return arr.larray
        full = arr._gathered()
        if like.is_distributed():
            counts, displs = like.counts_displs()
            r = like.comm.rank
            return full[displs[r]: displs[r] + counts[r]]
        return full

    def _partial_fit(self, x: DNDarray, y: DNDarray, classes: Optional[DNDarray], _refit: bool,
                     sample_weight: Optional[DNDarray]) -> "GaussianNB":
        if x.ndim != 2:
            raise ValueError("expected x to be a 2-D tensor, is {}-D".format(x.ndim))
        n_samples = x.gshape[0]
        if y.gshape[0] != n_samples:
            raise ValueError("y.shape[0] must match number of samples {}, is {}".format(n_samples, y.gshape[0]))
        if sample_weight is not None:
            if sample_weight.ndim != 1:
                raise ValueError("Sample weights must be 1D tensor")
            if sample_weight.gshape != (n_samples,):
                raise ValueError("sample_weight.shape == {}, expected {}!".format(sample_weight.shape, (n_samples,)))
        X = x.larray if x.larray.is_floating_point() else x.larray.double()
        dt = X.dtype
        self._epsilon = self.var_smoothing * float(ht.var(x, axis=0).max().item())
        if _refit:
            self.classes_ = None
        first = getattr(self, "classes_", None) is None
        if first:
            if classes is None:
                raise ValueError("classes must be passed on the first call to partial_fit.")
            cl = classes._gathered() if classes.is_distributed() else classes.larray
            self.classes_ = ht.array(cl, device=x.device, comm=x.comm)
            n_classes, n_features = cl.numel(), x.gshape[1]
            self.theta_ = ht.zeros((n_classes, n_features), dtype=ht.types.canonical_heat_type(dt), device=x.device,
                                   comm=x.comm)
            self.sigma_ = ht.zeros((n_classes, n_features), dtype=ht.types.canonical_heat_type(dt), device=x.device,
                                   comm=x.comm)
            self.class_count_ = ht.zeros((n_classes,), dtype=ht.float64, device=x.device, comm=x.comm)
            if self.priors is not None:
                pri = self.priors if isinstance(self.priors, DNDarray) else ht.array(self.priors, device=x.device)
                if len(pri) != n_classes:
                    raise ValueError("Number of priors must match number of classes.")
                if abs(float(pri.sum().item()) - 1.0) > 1e-6:
                    raise ValueError("The sum of the priors should be 1.")
                if bool((pri < 0).any().item()):
                    raise ValueError("Priors must be non-negative.")
                self.class_prior_ = pri
        else:
            if classes is not None:
                cl_new = classes._gathered() if classes.is_distributed() else classes.larray
                if cl_new.numel() != self.classes_.larray.numel() or not bool(
                        (cl_new.to(self.classes_.larray.device) == self.classes_.larray).all()):
                    raise ValueError("classes={} is not the same as on the last call to partial_fit, was {}".format(
                        cl_new.tolist(), self.classes_.larray.tolist()))
            if x.gshape[1] != self.theta_.gshape[1]:
                raise ValueError("Number of features {} does not match previous data {}.".format(
                    x.gshape[1], self.theta_.gshape[1]))
            self.sigma_.larray -= self._epsilon
        cl = self.classes_.larray
        yl = self._local_rows(y, x).to(cl.dtype).to(X.device)
        idx = torch.searchsorted(cl.contiguous(), yl.contiguous())
        bad = (idx >= cl.numel()) | (cl[idx.clamp(max=cl.numel() - 1)] != yl)
        any_bad = bool(bad.any()) if yl.numel() else False
        if x.is_distributed():
            # every rank must raise together (a lone raise would leave the others in a collective)
            any_bad = bool(x.comm.allreduce(int(any_bad), MPI.MAX))
        if any_bad:
            raise ValueError("The target label(s) {} in y do not exist in the initial classes {}".format(
                torch.unique(yl[bad]).tolist() if yl.numel() else [], cl.tolist()))
        k = cl.numel()
        f = X.shape[1]
        w = self._local_rows(sample_weight, x).to(torch.float64) if sample_weight is not None else \
            torch.ones(X.shape[0], dtype=torch.float64, device=X.device)
        Xd = X.to(torch.float64)
        # pass 1: weighted counts and sums -> means
        cnt = torch.zeros(k, dtype=torch.float64, device=X.device).index_add_(0, idx, w)
        sums = torch.zeros(k, f, dtype=torch.float64, device=X.device).index_add_(0, idx, Xd * w.unsqueeze(1))
        packed = torch.cat([cnt, sums.reshape(-1)])
        if x.is_distributed():
            x.comm.Allreduce(MPI.IN_PLACE, packed, MPI.SUM)
        cnt, sums = packed[:k], packed[k:].reshape(k, f)
        mu = sums / cnt.clamp(min=1e-300).unsqueeze(1)
        # pass 2: weighted squared deviations
        dev = (Xd - mu[idx]) ** 2 * w.unsqueeze(1)
        m2 = torch.zeros(k, f, dtype=torch.float64, device=X.device).index_add_(0, idx, dev)
        if x.is_distributed():
            x.comm.Allreduce(MPI.IN_PLACE, m2, MPI.SUM)
        # Chan merge with the previous state
        n_old = self.class_count_.larray.to(torch.float64)
        mu_old = self.theta_.larray.to(torch.float64)
        var_old = self.sigma_.larray.to(torch.float64)
        n_tot = n_old + cnt
        safe = n_tot.clamp(min=1e-300).unsqueeze(1)
        mu_new = (n_old.unsqueeze(1) * mu_old + cnt.unsqueeze(1) * mu) / safe
        m2_old = var_old * n_old.unsqueeze(1)
        m2_tot = m2_old + m2 + (n_old * cnt / n_tot.clamp(min=1e-300)).unsqueeze(1) * (mu_old - mu) ** 2
        var_new = m2_tot / safe
        upd = (cnt > 0).unsqueeze(1)
        self.theta_.larray = torch.where(upd, mu_new, mu_old).to(dt)
        self.sigma_.larray = (torch.where(upd, var_new, var_old) + self._epsilon).to(dt)
        self.class_count_.larray = n_tot.to(self.class_count_.larray.dtype)
        if self.priors is None:
            self.class_prior_ = ht.array((n_tot / n_tot.sum()).to(torch.float64), device=x.device, comm=x.comm)
        return self

    # ----------------------------------------------------------------- prediction
    def _joint_log_likelihood(self, x: DNDarray) -> DNDarray:
        if not isinstance(x, DNDarray):
            raise ValueError("input needs to be a ht.DNDarray, but was {}".format(type(x)))
        X = x.larray if x.larray.is_floating_point() else x.larray.double()
        theta = self.theta_.larray.to(X.dtype)
        sigma = self.sigma_.larray.to(X.dtype)
        prior = self.class_prior_.larray.to(X.dtype)
        n_ij = -0.5 * torch.sum(torch.log(2.0 * torch.pi * sigma), 1)                     # [k]
        quad = ((X.unsqueeze(1) - theta.unsqueeze(0)) ** 2 / sigma.unsqueeze(0)).sum(2)  # [m, k]
        jll = torch.log(prior).unsqueeze(0) + n_ij.unsqueeze(0) - 0.5 * quad
        return DNDarray(jll, (x.gshape[0], theta.shape[0]), ht.types.canonical_heat_type(jll.dtype), x.split,
                        x.device, x.comm, x.balanced)

    def logsumexp(self, a: DNDarray, axis=None, b: Optional[DNDarray] = None, keepdim: bool = False,
                  return_sign: bool = False) -> DNDarray:
        """Numerically stable ``log(sum(exp(a)))`` along ``axis``."""
        if b is not None:
            raise NotImplementedError("Not implemented for weighted logsumexp")
        if return_sign:
            raise NotImplementedError("Not implemented for return_sign")
        a_max = ht.max(a, axis=axis, keepdim=True)
        s = ht.sum(ht.exp(a - a_max), axis=axis, keepdim=keepdim)
        out = ht.log(s)
        if not keepdim:
            a_max = ht.squeeze(a_max, axis=axis)
        return out + a_max

    def predict(self, x: DNDarray) -> DNDarray:
        jll = self._joint_log_likelihood(x)
        idx = torch.argmax(jll.larray, dim=1)
        lab = self.classes_.larray[idx]
        return DNDarray(lab, (x.gshape[0],), self.classes_.dtype, x.split, x.device, x.comm, x.balanced)

    def predict_log_proba(self, x: DNDarray) -> DNDarray:
        jll = self._joint_log_likelihood(x)
        t = jll.larray
        norm = torch.logsumexp(t, dim=1, keepdim=True)
        return DNDarray(t - norm, jll.gshape, jll.dtype, jll.split, jll.device, jll.comm, jll.balanced)

    def predict_proba(self, x: DNDarray) -> DNDarray:
        return ht.exp(self.predict_log_proba(x))
