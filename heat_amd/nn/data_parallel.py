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


class _Done:
    """Completed request (world of one)."""

    def Wait(self) -> None:
        pass


class _Bucket:
    def __init__(self, params: List[torch.nn.Parameter]):
        self.params = params
        self.ready = 0
        self.reported = set()
        self.flat = None
        self.req = None

    def reset(self) -> None:
        self.ready = 0
        self.reported = set()
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
        self._callback_queued = False

    # ---------------------------------------------------------------- gradient synchronisation
    def _fire(self, b: _Bucket) -> None:
        """Launch the (async) all-reduce of one bucket. Parameters that produced no gradient on
        this rank contribute zeros, so a bucket is never left waiting for a gradient that will not
        come (reference: per-parameter hooks, ``nn/data_parallel.py:223-278``, average exactly the
        parameters that received a gradient)."""
        grads = [q.grad.reshape(-1) if (id(q) in b.reported and q.grad is not None)
                 else torch.zeros(q.numel(), device=q.device, dtype=q.dtype) for q in b.params]
        flat = torch.cat(grads).to(self.grad_dtype)  # a copy: a zero_grad() before the deferred
        flat.mul_(1.0 / self.comm.size)              # update cannot erase it
        b.flat = flat
        b.req = self.comm.Iallreduce(MPI.IN_PLACE, flat, MPI.SUM) if self.comm.is_distributed() else _Done()

    def _on_backward_end(self) -> None:
        """Queued on the autograd engine by the first gradient hook of a backward pass: buckets
        with a parameter that received no gradient are flushed here, in bucket order (the same on
        every rank as long as every rank uses the same parameters - the reference's and DDP's
        contract), while the gradients are still in place."""
        self._callback_queued = False
        for b in self._buckets:
            if b.req is None and b.reported:
                self._fire(b)

    def _grad_ready(self, p: torch.nn.Parameter) -> None:
        if not self.module.training:
            return
        if not (self.comm.is_distributed() or not self.blocking_parameter_updates):
            return  # world of one, blocking: the local gradient is the average
        b = self._buckets[self._bucket_of[id(p)]]
        self._pending = True
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._on_backward_end)
        if id(p) in b.reported:
            # second backward before the update (gradient accumulation): the flush in
            # _finish_gradient_sync re-sends the accumulated gradient
            if b.req is not None:
                b.req.Wait()
                b.req, b.flat = None, None
            return
        b.reported.add(id(p))
        b.ready += 1
        if b.ready == len(b.params):
            self._fire(b)

    @torch.no_grad()
    def _finish_gradient_sync(self, inplace: bool = True) -> None:
        if not self._pending:
            return
        # normally done at the end of backward already (_on_backward_end)
        for b in self._buckets:
            if b.req is None and b.reported:
                self._fire(b)
        for b in self._buckets:
            if b.req is None:
                b.reset()
                continue
            b.req.Wait()
            off = 0
            for q in b.params:
                n = q.numel()
                if id(q) in b.reported:
                    g = b.flat[off: off + n].reshape(q.shape).to(q.dtype)
                    if q.grad is None or not inplace:
                        q.grad = g.clone()
                    else:
                        q.grad.copy_(g)
                # a parameter without a gradient keeps grad None (the optimizer skips it, as in
                # the reference where no hook fires for it)
                off += n
            b.reset()
        self._pending = False

    def _deferred_update(self) -> None:
        """Non-blocking mode: apply the previous step's averaged gradients and optimizer step at
        the start of the next forward. The ``.grad`` the user left (usually None after
        ``zero_grad()``) is restored afterwards, so the coming backward does not accumulate onto
        the previous step's average (the reference's hooks likewise keep the averaged gradient
        out of the local accumulation, ``nn/data_parallel.py:255-276``)."""
        if not self._pending and not any(o.update_next for o in self._dp_optimizers):
            return
        stash = [(q, q.grad) for q in self.module.parameters()]
        self._finish_gradient_sync(inplace=False)
        for o in self._dp_optimizers:
            if o.update_next:
                o.torch_optimizer.step()
                o.update_next = False
        for q, g in stash:
            q.grad = g

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
