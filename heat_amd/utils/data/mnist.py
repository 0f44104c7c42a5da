"""MNIST as a distributed Dataset (reference ``heat/utils/data/mnist.py``: ``MNISTDataset`` 16).

The reference wraps torchvision; here the standard IDX files (``train-images-idx3-ubyte`` ...,
optionally gzipped) are parsed directly, so no torchvision is needed. Nothing is downloaded."""
from __future__ import annotations

import gzip
import os
from typing import Callable, Optional

import numpy as np
import torch

from ... import core as ht
from .datatools import Dataset, dataset_ishuffle, dataset_shuffle

__all__ = ["MNISTDataset"]


def _read_idx(path: str) -> np.ndarray:
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as f:
        data = f.read()
    ndim = data[3]
    dims = [int.from_bytes(data[4 + 4 * i: 8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def _find(root: str, stem: str) -> str:
    for d in (root, os.path.join(root, "MNIST", "raw"), os.path.join(root, "raw")):
        for ext in ("", ".gz"):
            p = os.path.join(d, stem + ext)
            if os.path.exists(p):
                return p
    raise FileNotFoundError("MNIST file {} not found under {} (no download is attempted)".format(stem, root))


class MNISTDataset(Dataset):
    """MNIST images/targets split along the sample axis across ranks."""

    def __init__(self, root: str, train: bool = True, transform: Optional[Callable] = None,
                 target_transform: Optional[Callable] = None, download: bool = False, split: int = 0,
                 ishuffle: bool = False, test_set: bool = False):
        if download:
            raise RuntimeError("downloading is not supported; place the IDX files under root")
        prefix = "train" if train else "t10k"
        imgs = _read_idx(_find(root, prefix + "-images-idx3-ubyte"))
        lbls = _read_idx(_find(root, prefix + "-labels-idx1-ubyte"))
        array = ht.array(torch.from_numpy(imgs.copy()), split=split)
        targets = ht.array(torch.from_numpy(lbls.astype(np.int64)), split=split)
        super().__init__(array, transforms=transform, ishuffle=ishuffle, test_set=test_set)
        self.httargets = targets
        self.targets = targets.larray[: self.data.shape[0]]
        self.target_transform = target_transform

    def __getitem__(self, index):
        img = self.data[index].float().div(255.0).unsqueeze(0)
        if self.transforms:
            img = self.transforms[0](img)
        target = self.targets[index]
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, target

    def Shuffle(self):
        if not self.test_set:
            dataset_shuffle(self, [["data", "htdata"], ["targets", "httargets"]])

    def Ishuffle(self):
        if not self.test_set:
            dataset_ishuffle(self, [["data", "htdata"], ["targets", "httargets"]])
