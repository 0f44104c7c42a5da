"""Optimizer utilities (reference ``heat/optim/utils.py``: ``DetectMetricPlateau`` 14 with
``get_state/set_state`` 72/89 for checkpointing, ``test_if_improving`` 117)."""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch

__all__ = ["DetectMetricPlateau"]


class DetectMetricPlateau:
    """Detect when a metric stops improving (adapted from ReduceLROnPlateau's bookkeeping)."""

    def __init__(self, mode: Optional[str] = "min", patience: Optional[int] = 10, threshold: Optional[float] = 1e-4,
                 threshold_mode: Optional[str] = "rel", cooldown: Optional[int] = 0):
        self.patience = patience
        self.cooldown = cooldown
        self.cooldown_counter = 0
        self.mode = mode
        self.threshold = threshold
        self.threshold_mode = threshold_mode
        self.best = None
        self.num_bad_epochs = None
        self.mode_worse = None
        self.last_epoch = 0
        self._init_is_better(mode=mode, threshold=threshold, threshold_mode=threshold_mode)
        self.reset()

    _STATE = ("patience", "cooldown", "cooldown_counter", "mode", "threshold", "threshold_mode", "best",
              "num_bad_epochs", "mode_worse", "last_epoch")

    def get_state(self) -> Dict:
        """Checkpointable state."""
        return {k: getattr(self, k) for k in self._STATE}

    def set_state(self, dic: Dict) -> None:
        for k in self._STATE:
            setattr(self, k, dic[k])

    def reset(self) -> None:
        self.best = self.mode_worse
        self.cooldown_counter = 0
        self.num_bad_epochs = 0

    def test_if_improving(self, metrics) -> bool:
        """True once the metric has not improved for more than ``patience`` epochs (a plateau)."""
        current = float(metrics)
        self.last_epoch += 1
        if self.is_better(current, self.best):
            self.best = current
            self.num_bad_epochs = 0
        else:
            self.num_bad_epochs += 1
        if self.in_cooldown:
            self.cooldown_counter -= 1
            self.num_bad_epochs = 0
        if self.num_bad_epochs > self.patience:
            self.cooldown_counter = self.cooldown
            self.num_bad_epochs = 0
            return True
        return False

    @property
    def in_cooldown(self) -> bool:
        return self.cooldown_counter > 0

    def is_better(self, a: float, best: float) -> bool:
        if self.mode == "min" and self.threshold_mode == "rel":
            return a < best * (1.0 - self.threshold)
        if self.mode == "min" and self.threshold_mode == "abs":
            return a < best - self.threshold
        if self.mode == "max" and self.threshold_mode == "rel":
            return a > best * (self.threshold + 1.0)
        return a > best + self.threshold

    def _init_is_better(self, mode: str, threshold: float, threshold_mode: str) -> None:
        if mode not in ("min", "max"):
            raise ValueError("mode " + mode + " is unknown!")
        if threshold_mode not in ("rel", "abs"):
            raise ValueError("threshold mode " + threshold_mode + " is unknown!")
        self.mode_worse = math.inf if mode == "min" else -math.inf
        self.mode = mode
        self.threshold = threshold
        self.threshold_mode = threshold_mode
