"""
Streaming HDF5 datasets (reference ``heat/utils/data/partial_dataset.py``: ``PartialH5Dataset`` 32,
``PartialH5DataLoaderIter`` 224): only a window of the file is resident; a background thread
loads the next window while the current one is consumed. Uses ``h5py`` when installed, the
built-in HDF5 reader (``heat_amd.core._h5lite``) otherwise.
"""
from __future__ import annotations

import queue
import threading
from typing import Callable, List, Optional, Union

import torch
from torch.utils import data as torch_data

from ...core.communication import MPI_WORLD

from ...core import _h5lite

try:
    import h5py
except ImportError:  # optional dependency: fall back to the built-in reader
    h5py = None


def _open(path: str):
    return h5py.File(path, "r") if h5py is not None else _h5lite.open_file(path)

__all__ = ["PartialH5Dataset", "PartialH5DataLoaderIter", "queue_thread"]


def queue_thread(q: queue.Queue) -> None:
    """Worker loop of the loader threads: run ``func(*args)`` (or a bare callable) per queue item."""
    while True:
        item = q.get()
        try:
            if isinstance(item, tuple):
                item[0](*item[1:])
            else:
                item()
        finally:
            q.task_done()


class PartialH5Dataset(torch_data.Dataset):
    """Window over this rank's share of HDF5 datasets (``dataset_names``), ``initial_load`` rows
    resident, ``load_length`` rows fetched per background load."""

    def __init__(self, file: str, comm=MPI_WORLD, dataset_names: Union[str, List[str]] = "data",
                 transforms: List[Callable] = None, use_gpu: bool = True, validate_set: bool = False,
                 initial_load: int = 7000, load_length: int = 1000):
        self.ishuffle = False
        self.file = file
        self.comm = comm
        self.transforms = transforms if isinstance(transforms, (list, tuple)) else [transforms]
        self.gpu = use_gpu and torch.cuda.is_available()
        self.validate_set = validate_set
        self.dataset_names = [dataset_names] if isinstance(dataset_names, str) else list(dataset_names)
        with _open(file) as f:
            self.total_size = f[self.dataset_names[0]].shape[0]
        self.lcl_full_sz = self.total_size // comm.size
        self.local_data_start = self.lcl_full_sz * comm.rank
        self.local_data_end = self.local_data_start + self.lcl_full_sz
        self.load_initial = min(initial_load, self.lcl_full_sz)
        self.load_len = load_length
        self.loads_remaining = max(0, (self.lcl_full_sz - self.load_initial) // max(1, load_length))
        self._f = _open(file)
        self.next_start = self.local_data_start + self.load_initial
        for name in self.dataset_names:
            arr = torch.tensor(self._f[name][self.local_data_start: self.next_start])
            setattr(self, name, arr.cuda() if self.gpu else arr)
        self.length = self.load_initial
        self.load_thread = None
        self.io_queue = queue.Queue()

    def Shuffle(self):
        pass

    def Ishuffle(self):
        pass

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, index):
        items = [getattr(self, n)[index] for n in self.dataset_names]
        if self.transforms and self.transforms[0] is not None:
            items = [t(x) if t is not None else x for t, x in zip(self.transforms, items)]
        return items[0] if len(items) == 1 else tuple(items)

    def thread_replace_converted_batches(self):
        """Background loader: read the next window and queue it."""
        while self.loads_remaining > 0:
            end = min(self.next_start + self.load_len, self.local_data_end)
            chunk = [torch.tensor(self._f[n][self.next_start: end]) for n in self.dataset_names]
            self.io_queue.put(chunk)
            self.next_start = end
            self.loads_remaining -= 1


class PartialH5DataLoaderIter:
    """Iterator for :class:`PartialH5Dataset`: consumes resident rows while the next window loads."""

    def __init__(self, loader):
        self.loader = loader
        self.dataset = loader.dataset
        self._it = iter(loader.DataLoader)
        if self.dataset.loads_remaining > 0 and self.dataset.load_thread is None:
            self.dataset.load_thread = threading.Thread(target=self.dataset.thread_replace_converted_batches,
                                                        daemon=True)
            self.dataset.load_thread.start()

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        return self

    def __next__(self):
        try:
            return next(self._it)
        except StopIteration:
            if not self.dataset.io_queue.empty():
                chunk = self.dataset.io_queue.get()
                for n, c in zip(self.dataset.dataset_names, chunk):
                    setattr(self.dataset, n, c.cuda() if self.dataset.gpu else c)
                self.dataset.length = chunk[0].shape[0]
                self._it = iter(self.loader.DataLoader)
                return next(self._it)
            raise
