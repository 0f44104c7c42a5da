"""
Data-parallel optimizers (reference ``heat/optim/dp_optimizer.py``: ``DASO`` 46-832,
``DataParallelOptimizer`` 834-877).

``DataParallelOptimizer`` wraps a torch optimizer for :class:`heat_amd.nn.DataParallel`; the
gradient averaging itself is bucketed and overlapped with the backward pass by the module.

``DASO`` (Distributed Asynchronous and Selective Optimization) keeps the reference's phases and
skip schedule: node-local synchronisation every step (DDP over RCCL on the node's xGMI mesh),
global parameter averaging among the ranks with the same local rank every ``global_skip``
batches, received ``batches_to_wait`` batches later and merged as a weighted stale average.
Differences by design: the global payload is ONE flat bf16/fp16/fp32 buffer all-reduced in
``sending_chunk_size`` pieces on RCCL (bf16/fp16 sums are native to RCCL, no custom MPI op is
needed), and the node-local parameter broadcast is one coalesced broadcast.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple, Union

import torch
import torch.distributed as dist

from ..core.communication import MPI, MPI_WORLD, MPICommunication
from .utils import DetectMetricPlateau

__all__ = ["DataParallelOptimizer", "DASO"]


class DataParallelOptimizer:
    """Torch optimizer wrapper for :class:`heat_amd.nn.DataParallel`.

    Blocking: ``step()`` finishes the gradient all-reduces and steps immediately. Non-blocking:
    the step is deferred to the beginning of the next forward pass (communication overlaps the
    data loading of the next batch), like the reference.
    """

    def __init__(self, torch_optimizer: torch.optim.Optimizer, blocking: bool = False):
        self.torch_optimizer = torch_optimizer
        if not isinstance(blocking, bool):
            raise TypeError("blocking parameter must be a boolean, currently {}".format(type(blocking)))
        self.blocking_parameter_updates = blocking
        self.update_next = False
        self.params_ref = torch_optimizer.param_groups[0]["params"]
        self._dp_module = None

    def step(self) -> None:
        if self.blocking_parameter_updates:
            if self._dp_module is not None:
                self._dp_module._finish_gradient_sync()
            self.torch_optimizer.step()
        else:
            self.update_next = True

    def zero_grad(self) -> None:
        self.torch_optimizer.param_groups[0]["params"] = self.params_ref[:]
        self.torch_optimizer.zero_grad()


class DASO:
    """Hierarchical data-parallel optimizer (see module docstring and the reference's docs).

    Parameters follow the reference: ``local_optimizer``, ``total_epochs``, ``comm``,
    ``warmup_epochs``, ``cooldown_epochs``, ``scheduler``, ``stability_level``,
    ``max_global_skips``, ``sending_chunk_size``, ``downcast_type``, ``use_mpi_groups``,
    ``skip_reduction_factor``, ``local_skip_factor``, ``verbose``.
    """

    def __init__(self, local_optimizer: torch.optim.Optimizer, total_epochs: int, comm: MPICommunication = MPI_WORLD,
                 warmup_epochs: int = 4, cooldown_epochs: int = 4, scheduler=None, stability_level: float = 0.05,
                 max_global_skips: int = 8, sending_chunk_size: int = 10_000_000,
                 downcast_type: torch.dtype = torch.bfloat16, use_mpi_groups: bool = True,
                 skip_reduction_factor: int = 2, local_skip_factor: int = 4, verbose: bool = False):
        if scheduler is not None and not (isinstance(scheduler, type) or hasattr(scheduler, "step")):
            raise TypeError("scheduler must be None or a torch lr_scheduler (class), currently {}".format(
                type(scheduler)))
        self._check_types(local_optimizer, total_epochs, comm, warmup_epochs, cooldown_epochs, stability_level,
                          max_global_skips, sending_chunk_size, downcast_type, use_mpi_groups, skip_reduction_factor,
                          local_skip_factor, verbose)
        self.local_optimizer = local_optimizer
        self.params_ref = local_optimizer.param_groups[0]["params"]
        self.comm = comm
        self.verbose = verbose
        self.scheduler = scheduler
        self.cast_dtype = downcast_type
        self.module = None
        self.amp = False
        self.scaler = None
        # node topology: ranks [node * loc_gpus, ..., node * loc_gpus + loc_gpus - 1] share a node
        import os

        loc = int(os.environ.get("LOCAL_WORLD_SIZE", "0")) or max(1, torch.cuda.device_count())
        self.loc_gpus = max(1, min(loc, comm.size))
        if comm.size % self.loc_gpus:
            self.loc_gpus = 1
        self.nodes = comm.size // self.loc_gpus
        rank = comm.rank
        self.local_rank = rank % self.loc_gpus
        self.base_loc_ranks = list(range(0, comm.size, self.loc_gpus))
        reduced_comms, reduced_ranks = [], []
        for i in range(self.loc_gpus):
            lp_ranks = [j + i for j in self.base_loc_ranks]
            reduced_ranks.append(tuple(lp_ranks))
            reduced_comms.append(comm.Create_group(lp_ranks) if comm.size > 1 else comm)
        self.reduced_comms, self.reduced_ranks = reduced_comms, reduced_ranks
        node = rank // self.loc_gpus
        local_ranks = [node * self.loc_gpus + i for i in range(self.loc_gpus)]
        self.local_comm = None
        for nd in range(self.nodes):
            lr = [nd * self.loc_gpus + i for i in range(self.loc_gpus)]
            c = comm.Create_group(lr) if comm.size > 1 else comm
            if nd == node:
                self.local_comm = c
        self.local_ranks = local_ranks
        self.current_batch, self.last_batch = 0, None
        self._prev_params = []
        self.epoch = 0
        self._send_mod, self._send_mod_m1 = 0, None
        self.global_skip = 0
        self.local_skip = 0
        self.batches_to_wait = 0
        self.max_gs = max_global_skips
        self.warmup_epochs = warmup_epochs
        self.cooldown_epochs = cooldown_epochs
        self.total_epochs = total_epochs
        self.skip_reduction_factor = skip_reduction_factor
        self.local_skip_factor = local_skip_factor
        self.stability = DetectMetricPlateau(patience=2, threshold=stability_level)
        self._gs8_waits = 3
        self._gs8_waited = 0
        self.split_val = sending_chunk_size
        self.print0("Finished DASO init")

    @staticmethod
    def _check_types(local_optimizer, total_epochs, comm, warmup_epochs, cooldown_epochs, stability_level,
                     max_global_skips, sending_chunk_size, downcast_type, use_mpi_groups, skip_reduction_factor,
                     local_skip_factor, verbose):
        if not isinstance(local_optimizer, torch.optim.Optimizer):
            raise TypeError("Local optimizer must be a torch optimizer object, currently {}".format(type(local_optimizer)))
        if not isinstance(comm, MPICommunication):
            raise TypeError("Comm object must be a ht.MPICommunication object, currently {}".format(type(comm)))
        for name, val in (("total_epochs", total_epochs), ("warmup_epochs", warmup_epochs),
                          ("cooldown_epochs", cooldown_epochs), ("max_global_skips", max_global_skips),
                          ("sending_chunk_size", sending_chunk_size), ("skip_reduction_factor", skip_reduction_factor),
                          ("local_skip_factor", local_skip_factor)):
            if not isinstance(val, int) or isinstance(val, bool):
                raise TypeError("{} must be an int, currently {}".format(name, type(val)))
            if val < 0:
                raise ValueError("{} must be >= 0, currently {}".format(name, val))
        if not isinstance(stability_level, float):
            raise TypeError("stability_level must be a float, currently {}".format(type(stability_level)))
        if downcast_type not in (torch.bfloat16, torch.half, torch.float):
            raise TypeError("downcast_type must be in [torch.bfloat16, torch.half, torch.float], currently "
                             "{}".format(downcast_type))
        if not isinstance(use_mpi_groups, bool) or not isinstance(verbose, bool):
            raise TypeError("use_mpi_groups and verbose must be bools")

    # ------------------------------------------------------------------ API
    def add_scaler(self, scaler) -> None:
        """Use a ``torch.amp.GradScaler`` in :meth:`step`."""
        self.scaler = scaler
        self.amp = True

    def set_model(self, model: torch.nn.Module) -> None:
        self.module = model

    def print0(self, *args, **kwargs) -> None:
        if self.comm.rank == 0 and self.verbose:
            print(*args, **kwargs)

    def reset(self) -> None:
        self.stability.reset()
        self.global_skip = 0
        self.local_skip = 0
        self.batches_to_wait = 0
        self.current_batch = 0
        self._prev_params = []
        self.epoch = 0
        self._gs8_waited = 0
        self.zero_grad()

    def zero_grad(self) -> None:
        self.local_optimizer.param_groups[0]["params"] = self.params_ref[:]
        self.local_optimizer.zero_grad()

    def epoch_loss_logic(self, loss: Union[torch.Tensor, int, float], loss_globally_averaged: bool = False) -> None:
        """Adapt global/local skips and staleness from the epoch's loss (warm-up, cycling, cool-down)."""
        if not loss_globally_averaged:
            val = float(loss.detach().float().mean()) if isinstance(loss, torch.Tensor) else float(loss)
            avg_loss = self.comm.allreduce(val, MPI.SUM) / self.comm.size
        else:
            avg_loss = float(loss)
        if self.epoch < self.warmup_epochs:
            self.global_skip = self.local_skip = self.batches_to_wait = 0
            self.print0("Warmup Phase, Global Skips: {}, Local Skips {}, Batches to wait: {}".format(
                self.global_skip, self.local_skip, self.batches_to_wait))
            return
        if self.warmup_epochs == self.epoch:
            self.global_skip, self.local_skip, self.batches_to_wait = 4, 1, 1
        if self.epoch >= self.total_epochs - self.cooldown_epochs:
            self.global_skip = self.local_skip = self.batches_to_wait = 0
            self.print0("Cooldown Phase")
            return
        if self.global_skip == self.max_gs and self.max_gs > 4:
            self._gs8_waited += 1
        stable = self.stability.test_if_improving(avg_loss)
        if stable and self.global_skip > 1:
            self.global_skip //= self.skip_reduction_factor
            self.local_skip //= self.skip_reduction_factor
            self.batches_to_wait -= 1
            if self.global_skip > 0:
                self.batches_to_wait = max(self.batches_to_wait, 1)
                self.local_skip = max(self.local_skip, 1)
            self._gs8_waited = 0
        elif self.global_skip == 1 and stable:
            self.global_skip = self.max_gs
            self.local_skip = self.max_gs // self.local_skip_factor
            self.batches_to_wait = self.max_gs // self.local_skip_factor
            self._gs8_waited = 0
        self.print0("Next Parameters: Global Skips: {}, Local Skips {}, Batches to wait: {}, loss {:.4f}".format(
            self.global_skip, self.local_skip, self.batches_to_wait, avg_loss))

    # ------------------------------------------------------------------ synchronisation
    def _named_trainable(self):
        mod = self.module.module if hasattr(self.module, "module") and not isinstance(
            self.module, torch.nn.Sequential) else self.module
        return [(n, p) for n, p in self.module.named_parameters() if p.requires_grad]

    @torch.no_grad()
    def _pack(self, cast: bool) -> Tuple[torch.Tensor, Dict]:
        params = self._named_trainable()
        shapes, off = {}, 0
        for name, p in params:
            shapes[name] = (p.shape, slice(off, off + p.numel()), p.dtype)
            off += p.numel()
        dtype = self.cast_dtype if cast else torch.float32
        flat = torch.empty(off, dtype=dtype, device=params[0][1].device if params else "cpu")
        for name, p in params:
            flat[shapes[name][1]] = p.detach().reshape(-1).to(dtype)
        return flat, shapes

    @torch.no_grad()
    def _gs_send_params(self, current_comm: MPICommunication, batches_to_wait: int) -> None:
        """Pack the parameters into ONE flat buffer and all-reduce it in chunks (async)."""
        cast = self.global_skip < 1
        flat, shapes = self._pack(cast)
        if torch.isnan(flat.float()).any():
            raise ValueError("NaNs in the parameters to be sent")
        n = flat.numel()
        chunks = max(1, math.ceil(n / self.split_val))
        reqs = []
        for c in range(chunks):
            piece = flat[c * self.split_val: (c + 1) * self.split_val]
            reqs.append(current_comm.Iallreduce(MPI.IN_PLACE, piece, MPI.SUM))
        self._prev_params.append([reqs, flat, shapes, batches_to_wait])

    @torch.no_grad()
    def _gs_rcv_update_params(self) -> None:
        """Merge the previously sent (now averaged) parameters with the current ones."""
        if self._send_mod_m1 is None:
            return
        prev_ranks = self.reduced_ranks[self._send_mod_m1]
        if self.comm.rank not in prev_ranks or len(self._prev_params) == 0:
            return
        reqs, flat, shapes, batches_between = self._prev_params.pop(0)
        for r in reqs:
            r.Wait()
        numer = batches_between * 2.0 if batches_between > 0 else 1.0
        denom = float(len(prev_ranks) + numer)
        factor = numer / denom
        rcv = flat.float() / denom
        for name, p in self._named_trainable():
            shp, sl, dt = shapes[name]
            p.mul_(factor)
            p.add_(rcv[sl].reshape(shp).to(dt))

    @torch.no_grad()
    def _gs_rcv_update_params_last_batch(self, current_ranks: Tuple) -> None:
        if len(self._prev_params) > 1:
            raise ValueError("length of previous params > 1! {}".format(len(self._prev_params)))
        reqs, flat, shapes, _ = self._prev_params.pop(0)
        for r in reqs:
            r.Wait()
        rcv = flat.float() / float(len(current_ranks))
        for name, p in self._named_trainable():
            shp, sl, dt = shapes[name]
            p.copy_(rcv[sl].reshape(shp).to(dt))

    @torch.no_grad()
    def _local_update(self, sending_process) -> None:
        """Broadcast the parameters of the node-local rank ``sending_process`` inside the node."""
        if sending_process is None or self.loc_gpus == 1 or self.local_comm is None:
            return
        flat, shapes = self._pack(False)
        self.local_comm.Bcast(flat, root=sending_process)
        for name, p in self._named_trainable():
            shp, sl, dt = shapes[name]
            p.copy_(flat[sl].reshape(shp).to(dt))

    @torch.no_grad()
    def _global_sync(self, batches_to_wait: int) -> None:
        current_comm = self.reduced_comms[self._send_mod]
        current_ranks = self.reduced_ranks[self._send_mod]
        # merge the previous (stale) global average BEFORE posting the new one: with one rank per
        # node the sending group repeats, and receiving after sending would consume the buffer
        # just posted (the reference orders it the other way, which is only safe for loc_gpus > 1)
        if self.batches_to_wait != 0:
            self._gs_rcv_update_params()
            self._local_update(self._send_mod_m1)
        if self.comm.rank in current_ranks:
            self._gs_send_params(current_comm, batches_to_wait)
        if self.current_batch == self.last_batch or self.batches_to_wait == 0:
            if self.comm.rank in current_ranks:
                self._gs_rcv_update_params_last_batch(current_ranks)
            self._local_update(self._send_mod)
            self._send_mod_m1 = None
            if self.current_batch == self.last_batch:
                self._send_mod = 0
                self.epoch += 1
                self.current_batch = 0
            else:
                self.current_batch += 1
                self._send_mod = self._send_mod + 1 if self._send_mod <= self.loc_gpus - 2 else 0
        else:
            self.current_batch += 1
            self._send_mod_m1 = self._send_mod
            self._send_mod = self._send_mod + 1 if self._send_mod <= self.loc_gpus - 2 else 0

    def _start_local_sync(self) -> None:
        if hasattr(self.module, "require_backward_grad_sync"):
            self.module.require_backward_grad_sync = True

    def _stop_local_sync(self) -> None:
        if hasattr(self.module, "require_backward_grad_sync"):
            self.module.require_backward_grad_sync = False

    def step(self) -> None:
        """Local optimizer step plus the global/local synchronisation schedule.
        ``self.last_batch`` must be set to the number of batches per epoch."""
        if self.last_batch is None:
            raise ValueError("self.last_batch must be set as the number of batches (len(dataloader))")
        if self.amp:
            self.scaler.step(self.local_optimizer)
            self.scaler.update()
        elif self.scheduler is None:
            self.local_optimizer.step()
        else:
            self.scheduler.step()
        batch = self.current_batch
        next_batch = batch + 1
        gs, ls = self.global_skip, self.local_skip
        gmod = batch % gs if gs > 0 else 0
        btw = self.batches_to_wait if self.batches_to_wait + batch <= self.last_batch else self.last_batch - batch
        if batch == self.last_batch or gmod == 0:
            return self._global_sync(btw)
        if gs > 0 and next_batch % gs == 0:
            self._start_local_sync()
            self.current_batch += 1
            return
        if gmod < btw:
            self.current_batch += 1
            if next_batch == self.last_batch:
                self._start_local_sync()
            return
        if gmod == btw:
            self._gs_rcv_update_params()
            self._local_update(self._send_mod_m1)
            if ls > 1:
                self._stop_local_sync()
        if ls == 1 and next_batch != self.last_batch:
            self.current_batch += 1
            self._start_local_sync()
            return
        lmod = batch % ls if ls > 0 else 0
        if lmod == 0:
            self._stop_local_sync()
        elif next_batch % ls == 0:
            self._start_local_sync()
        if next_batch == self.last_batch:
            self._start_local_sync()
        self.current_batch += 1
