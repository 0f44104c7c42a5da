"""Estimator base classes and mixins (reference ``heat/core/base.py``: ``BaseEstimator`` 13,
``ClassificationMixin`` 98, ``ClusteringMixin`` 145, ``RegressionMixin`` 176, ``is_*`` 221-258)."""
from __future__ import annotations

import inspect
import json
from typing import Dict, List

from .dndarray import DNDarray

__all__ = ["BaseEstimator", "ClassificationMixin", "ClusteringMixin", "RegressionMixin", "is_classifier",
           "is_estimator", "is_clusterer", "is_regressor"]


class BaseEstimator:
    """Base of all estimators: constructor parameters are introspected for get/set_params."""

    @classmethod
    def _parameter_names(cls) -> List[str]:
        init = cls.__init__
        if init is object.__init__:
            return []
        sig = inspect.signature(init)
        return [p.name for p in sig.parameters.values() if p.name != "self" and p.kind == p.POSITIONAL_OR_KEYWORD]

    def get_params(self, deep: bool = True) -> Dict[str, object]:
        params = {}
        for key in self._parameter_names():
            value = getattr(self, key)
            if deep and hasattr(value, "get_params"):
                value = value.get_params()
            params[key] = value
        return params

    def __repr__(self, indent: int = 1) -> str:
        return "{}({})".format(self.__class__.__name__, json.dumps(self.get_params(), indent=4, default=str))

    def set_params(self, **params) -> "BaseEstimator":
        if not params:
            return self
        names = self._parameter_names()
        for key, value in params.items():
            if key not in names:
                raise ValueError("Invalid parameter {} for estimator {}. Check the list of available parameters with "
                                 "`estimator.get_params().keys()`.".format(key, self))
            if isinstance(value, dict):
                getattr(self, key).set_params(**value)
            else:
                setattr(self, key, value)
        return self


class ClassificationMixin:
    """Mixin for classifiers."""

    def fit(self, x: DNDarray, y: DNDarray):
        raise NotImplementedError()

    def fit_predict(self, x: DNDarray, y: DNDarray) -> DNDarray:
        self.fit(x, y)
        return self.predict(x)

    def predict(self, x: DNDarray) -> DNDarray:
        raise NotImplementedError()


class ClusteringMixin:
    """Mixin for clusterers."""

    def fit(self, x: DNDarray):
        raise NotImplementedError()

    def fit_predict(self, x: DNDarray) -> DNDarray:
        self.fit(x)
        return self.predict(x)


class RegressionMixin:
    """Mixin for regressors."""

    def fit(self, x: DNDarray, y: DNDarray):
        raise NotImplementedError()

    def fit_predict(self, x: DNDarray, y: DNDarray) -> DNDarray:
        self.fit(x, y)
        return self.predict(x)

    def predict(self, x: DNDarray) -> DNDarray:
        raise NotImplementedError()


def is_classifier(estimator: object) -> bool:
    """True when ``estimator`` is a ClassificationMixin."""
    return isinstance(estimator, ClassificationMixin)


def is_estimator(estimator: object) -> bool:
    """True when ``estimator`` is a BaseEstimator."""
    return isinstance(estimator, BaseEstimator)


def is_clusterer(estimator: object) -> bool:
    """True when ``estimator`` is a ClusteringMixin."""
    return isinstance(estimator, ClusteringMixin)


def is_regressor(estimator: object) -> bool:
    """True when ``estimator`` is a RegressionMixin."""
    return isinstance(estimator, RegressionMixin)
