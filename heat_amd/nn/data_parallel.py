"""
Data-parallel training (reference ``heat/nn/data_parallel.py``: ``DataParallel`` 21 with blocking
(223-241) and non-blocking (243-297) gradient hooks, ``DataParallelMultiGPU`` 314).

The reference all-reduces every parameter tensor separately in fp32. Here gradients are grouped
into ~``bucket_cap_mb`` flat buckets in backward order; a bucket's all-reduce (RCCL over xGMI, async)
is launched from the post-accumulate-grad hook of its last gradient, so communication overlaps
the rest of the backward pass. Blocking mode waits in ``optimizer.step()``; non-blocking mode
applies the averaged gradients and the optimizer step at the start of the next forward pass
(the reference's deferred update), overlapping the all-reduce with data loading.
"""
from __future__ import annotations

import warnings
from typing import Any, List, Optional, Tuple, Union

import torch
import torch.distributed as dist
import torch.nn as tnn

from ..core.communication import MPI, MPI_WORLD, MPICommunication
from .. import optim

__all__ = ["DataParallel", "DataParallelMultiGPU"]


class _Bucket:
    def __init__(self, params: List[torch.nn.Parameter]):
        self.params = params
        self.ready = 0
        self.flat = None
        self.req = None


class DataParallel(tnn.Module):
    """Replicate ``module`` on every rank and average gradients across ``comm``.

    Parameters: ``module``, ``comm``, ``optimizer`` (one or more
    :class:`heat_amd.optim.DataParallelOptimizer`), ``blocking_parameter_updates``,
    ``bucket_cap_mb`` (gradient bucket size), ``grad_dtype`` (wire dtype, fp32 default; bf16 halves
    the traffic).
    """

    def __init__(self, module: torch.nn.Module, comm: MPICommunication, optimizer, blocking_parameter_updates: bool = False,
                 bucket_cap_mb: float = 25.0, grad_dtype: torch.dtype = torch.float32):
        if isinstance(optimizer, optim.DASO):
            raise TypeError("For use with DASO please use DataParallelMultiGPU instead of DataParallel")
        super().__init__()
        self.module = module
        self.comm = comm
        self.blocking_parameter_updates = blocking_parameter_updates
        self.grad_dtype = grad_dtype
        opts = optimizer if isinstance(optimizer, (list, tuple)) else [optimizer]
        for o in opts:
            if not isinstance(o, optim.DataParallelOptimizer):
                raise TypeError("optimizers must be optim.DataParallelOptimizer")
        if not self.blocking_parameter_updates:
            if len(opts) > 1 or list(module.parameters()) != opts[0].torch_optimizer.param_groups[0]["params"]:
                self.blocking_parameter_updates = True
                warnings.warn("Usage of more than one DataParallelOptimizer causes fallback on blocking "
                              "communication during parameter updates.", stacklevel=2)
        self._dp_optimizers = list(opts)
        for o in opts:
            o.blocking_parameter_updates = self.blocking_parameter_updates
            o._dp_module = self
        # identical initial parameters on every rank: seeded reset (reference) + broadcast from 0
        torch.random.manual_seed(2147483646)
        self.module.apply(self._reset_parameters)
        with torch.no_grad():
            for p in self.module.parameters():
                if comm.is_distributed():
                    comm.Bcast(p.data, root=0)
        # gradient buckets in (approximate) backward order = reverse registration order
        params = [p for p in self.module.parameters() if p.requires_grad]
        cap = int(bucket_cap_mb * (1 << 20))
        self._buckets: List[_Bucket] = []
        cur, size = [], 0
        for p in reversed(params):
            cur.append(p)
            size += p.numel() * 4
            if size >= cap:
                self._buckets.append(_Bucket(cur))
                cur, size = [], 0
        if cur:
            self._buckets.append(_Bucket(cur))
        self._bucket_of = {}
        for bi, b in enumerate(self._buckets):
            for p in b.params:
                self._bucket_of[id(p)] = bi
        self._hooks = [p.register_post_accumulate_grad_hook(self._grad_ready) for p in params]
        self._pending = False

    # ---------------------------------------------------------------- gradient synchronisation
    def _grad_ready(self, p: torch.nn.Parameter) -> None:
        if not self.comm.is_distributed() or not self.module.training:
            return
        b = self._buckets[self._bucket_of[id(p)]]
        b.ready += 1
        if b.ready == len(b.params):
            grads = [q.grad.reshape(-1) if q.grad is not None else torch.zeros(q.numel(), device=q.device,
                                                                              dtype=q.dtype) for q in b.params]
            flat = torch.cat(grads).to(self.grad_dtype)
            flat.mul_(1.0 / self.comm.size)
            b.flat = flat
            b.req = self.comm.Iallreduce(MPI.IN_PLACE, flat, MPI.SUM)
            b.ready = 0
            self._pending = True

    @torch.no_grad()
    def _finish_gradient_sync(self) -> None:
        if not self._pending:
            return
        for b in self._buckets:
            if b.req is None:
                continue
            b.req.Wait()
            off = 0
            for q in b.params:
                n = q.numel()
                g = b.flat[off: off + n].reshape(q.shape).to(q.dtype)
                if q.grad is None:
                    q.grad = g.clone()
                else:
                    q.grad.copy_(g)
                off += n
            b.req = None
            b.flat = None
        self._pending = False

    def _deferred_update(self) -> None:
        self._finish_gradient_sync()
        for o in self._dp_optimizers:
            if o.update_next:
                o.torch_optimizer.step()
                o.update_next = False

    def __setattr__(self, name: str, value: Any) -> None:
        # leaving training mode finalises a pending (non-blocking) update, like the reference
        if name == "training" and not value and "_dp_optimizers" in self.__dict__ and \
                not self.__dict__.get("blocking_parameter_updates", True):
            self._deferred_update()
        super().__setattr__(name, value)

    def forward(self, *inputs, **kwargs):
        if not self.blocking_parameter_updates and self.module.training:
            self._deferred_update()
        return self.module(*inputs, **kwargs)

    @staticmethod
    def _reset_parameters(module: tnn.Module) -> None:
        if callable(getattr(module, "reset_parameters", None)):
            module.reset_parameters()


class DataParallelMultiGPU(tnn.Module):
    """Node-local data parallelism for :class:`heat_amd.optim.DASO`: the module is wrapped in
    ``DistributedDataParallel`` over the node's process group (RCCL over xGMI); global
    synchronisation is done by DASO itself."""

    def __init__(self, module: torch.nn.Module, optimizer, comm: MPICommunication = MPI_WORLD):
        super().__init__()
        if not isinstance(optimizer, optim.DASO):
            raise TypeError("optimizer must be a DASO optimizer")
        self.comm = comm
        if optimizer.loc_gpus > 1 and optimizer.local_comm is not None and optimizer.local_comm.group is not None:
            p0 = next(module.parameters(), None)
            dev = p0.device.index if p0 is not None and p0.is_cuda else None
            module = tnn.parallel.DistributedDataParallel(module, device_ids=[dev] if dev is not None else None,
                                                          process_group=optimizer.local_comm.group)
        self.module = module
        # identical initial parameters everywhere
        torch.random.manual_seed(2147483646)
        self.module.apply(DataParallel._reset_parameters)
        with torch.no_grad():
            if comm.is_distributed():
                for p in self.module.parameters():
                    comm.Bcast(p.data, root=0)
        optimizer.set_model(self.module)

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)
