"""
Data loaders for DNDarrays (reference ``heat/utils/data/datatools.py``: ``DataLoader`` 16,
``Dataset`` 143, ``dataset_shuffle`` 246, ``dataset_ishuffle`` 301, ``dataset_irecv`` 343).

Between epochs half of every rank's samples move to the next rank on a ring (one batched
send/recv pair over RCCL/gloo), then the local samples are permuted; the non-blocking variant
posts the exchange at the start of an epoch and completes it at the next.
"""
from __future__ import annotations

from typing import Callable, Iterator, List, Optional, Union

import torch

from ...parallel import staging as _SD
import torch.distributed as dist
from torch.utils import data as torch_data

from ...core.dndarray import DNDarray
from . import partial_dataset

__all__ = ["DataLoader", "Dataset", "dataset_shuffle", "dataset_ishuffle", "dataset_irecv"]


class DataLoader:
    """Iterable over the local part of a (distributed) dataset with a global ring shuffle between
    epochs. Wraps ``torch.utils.data.DataLoader`` (random sampler) for batching."""

    def __init__(self, dataset, batch_size: int = 1, num_workers: int = 0, collate_fn: Callable = None,
                 pin_memory: bool = False, drop_last: bool = False, timeout: Union[int, float] = 0,
                 worker_init_fn: Callable = None):
        if isinstance(dataset, DNDarray):
            dataset = Dataset(dataset)
        if not isinstance(dataset, (torch_data.Dataset, Dataset, partial_dataset.PartialH5Dataset)):
            raise TypeError("dataset must be a torch Dataset, heat Dataset, heat PartialH5Dataset, currently: {}"
                            .format(type(dataset)))
        self.dataset = dataset
        self.ishuffle = getattr(dataset, "ishuffle", False)
        if isinstance(dataset, partial_dataset.PartialH5Dataset):
            drop_last = True
        self.DataLoader = torch_data.DataLoader(dataset=dataset, batch_size=batch_size, shuffle=True,
                                                num_workers=num_workers, collate_fn=collate_fn, drop_last=drop_last,
                                                pin_memory=pin_memory, timeout=timeout, worker_init_fn=worker_init_fn)
        self._first_iter = True
        self.last_epoch = False

    def __iter__(self) -> Iterator:
        if isinstance(self.dataset, partial_dataset.PartialH5Dataset):
            return partial_dataset.PartialH5DataLoaderIter(self)
        self._full_dataset_shuffle_iter()
        return self.DataLoader.__iter__()

    def __len__(self) -> int:
        if isinstance(self.dataset, partial_dataset.PartialH5Dataset):
            # batches per epoch over the rank's share (len(dataset) is the whole file)
            bs = self.DataLoader.batch_size
            n = self.dataset.lcl_full_sz
            return n // bs if self.DataLoader.drop_last else -(-n // bs)
        return len(self.DataLoader)

    def _full_dataset_shuffle_iter(self):
        if not isinstance(self.dataset, Dataset):
            return
        if not self.ishuffle:
            if self._first_iter:
                self._first_iter = False
            else:
                self.dataset.Shuffle()
        else:
            if not self.last_epoch:
                self.dataset.Ishuffle()
            if self._first_iter:
                self._first_iter = False
            else:
                dataset_irecv(self.dataset)


class Dataset(torch_data.Dataset):
    """Dataset over the local block of a split DNDarray (every rank keeps the same number of
    samples; surplus rows are cut). Subclass and override ``__getitem__``/``Shuffle`` for targets."""

    def __init__(self, array: DNDarray, transforms: Optional[Union[List, Callable]] = None,
                 ishuffle: Optional[bool] = False, test_set: Optional[bool] = False):
        self.htdata = array
        self.comm = array.comm
        self.test_set = test_set
        split = array.split if array.split is not None else 0
        min_data_split = array.gshape[split] // array.comm.size if array.is_distributed() else array.gshape[split]
        self.lcl_half = min_data_split // 2
        sl = [slice(None)] * array.ndim
        sl[split] = slice(min_data_split)
        self._cut_slice = tuple(sl)
        self.data = array.larray[self._cut_slice]
        if not isinstance(transforms, (list, tuple)) and transforms is not None:
            transforms = [transforms]
        self.transforms = transforms
        self.ishuffle = ishuffle

    def __getitem__(self, index):
        if self.transforms:
            return self.transforms[0](self.data[index])
        return self.data[index]

    def __len__(self) -> int:
        return self.data.shape[0]

    def Shuffle(self):
        if not self.test_set:
            dataset_shuffle(dataset=self, attrs=[["data", "htdata"]])

    def Ishuffle(self):
        if not self.test_set:
            dataset_ishuffle(dataset=self, attrs=[["data", "htdata"]])


def _ring(comm):
    return (comm.rank + 1) % comm.size, (comm.rank - 1) % comm.size


def dataset_shuffle(dataset, attrs: List[list]):
    """Send the first half of the local samples to rank+1, receive rank-1's, permute locally."""
    comm = dataset.comm
    first = getattr(dataset, attrs[0][0])
    prm = torch.randperm(first.shape[0], device=first.device if first.is_cuda else "cpu")
    for data_attr, ht_attr in attrs:
        ld = getattr(dataset, data_attr)
        if comm.is_distributed():
            snd = ld[: dataset.lcl_half].clone()
            dest, src = _ring(comm)
            rcv = comm.sendrecv_tensor(snd, dest, tuple(snd.shape), src, dtype=snd.dtype, device=snd.device)
            ld = torch.cat([rcv, ld[dataset.lcl_half:]], dim=0)
        ld = ld[prm.to(ld.device)]
        setattr(dataset, data_attr, ld)
        if ht_attr is not None:
            ht = getattr(dataset, ht_attr)
            t = ht.larray
            t[dataset._cut_slice] = ld
    return dataset


def dataset_ishuffle(dataset, attrs: List[list]):
    """Non-blocking :func:`dataset_shuffle`: post the ring exchange; :func:`dataset_irecv` completes it."""
    comm = dataset.comm
    pending = []
    for data_attr, ht_attr in attrs:
        ld = getattr(dataset, data_attr)
        if not comm.is_distributed():
            continue
        snd = ld[: dataset.lcl_half].clone()
        dest, src = _ring(comm)
        rcv = torch.empty_like(snd)
        ops = [dist.P2POp(dist.isend, snd, comm._g(dest), comm.group),
               dist.P2POp(dist.irecv, rcv, comm._g(src), comm.group)]
        works = _SD.batch_isend_irecv(ops)
        pending.append((data_attr, ht_attr, works, snd, rcv))
    dataset._ishuffle_pending = pending
    return dataset


def dataset_irecv(dataset):
    """Complete a pending :func:`dataset_ishuffle` and permute the local samples."""
    pending = getattr(dataset, "_ishuffle_pending", [])
    prm = None
    for data_attr, ht_attr, works, snd, rcv in pending:
        for w in works:
            w.wait()
        ld = getattr(dataset, data_attr)
        ld = torch.cat([rcv, ld[dataset.lcl_half:]], dim=0)
        if prm is None:
            prm = torch.randperm(ld.shape[0])
        ld = ld[prm.to(ld.device)]
        setattr(dataset, data_attr, ld)
        if ht_attr is not None:
            getattr(dataset, ht_attr).larray[dataset._cut_slice] = ld
    dataset._ishuffle_pending = []
    return dataset
