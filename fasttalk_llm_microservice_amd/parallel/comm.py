"""Tensor-parallel communicator (RCCL over xGMI via torch.distributed).

``torch.distributed`` with ``backend="nccl"`` *is* RCCL on ROCm.  A TP group of
one process per GPU issues exactly two collectives per transformer layer (after
the row-parallel O and down projections) plus one
all-gather of vocab-sharded logits per step (X4).  Small decode-size messages
(≤ ``custom_max_bytes``) can go through :mod:`.custom_allreduce` (one-shot over
xGMI peer mappings) when it is enabled and initialised; everything else uses
RCCL.  On CPU (tests) the same code runs over ``gloo``.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


class TPComm:
    def __init__(self, group: Optional["dist.ProcessGroup"] = None, rank: int = 0,
                 world_size: int = 1):
        self.group = group
        self.rank = rank
        self.world_size = world_size
        self.custom = None  # CustomAllReduce, optional
        self.custom_max_bytes = 8 << 20
        self._host_staged: Optional[bool] = None

    @property
    def enabled(self) -> bool:
        return self.world_size > 1

    def _custom_on(self) -> bool:
        return self.custom is not None and not self.custom.failed

    def _via_host(self, x: torch.Tensor) -> bool:
        """gloo carries device tensors through host memory (ranks sharing one GPU in
        tests, where RCCL refuses duplicate devices); never graph-capturable."""
        if self._host_staged is None:
            self._host_staged = dist.get_backend(self.group) != "nccl"
        return self._host_staged and x.is_cuda

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.world_size == 1:
            return x
        if (self._custom_on() and x.is_cuda
                and x.numel() * x.element_size() <= self.custom_max_bytes
                and self.custom.can_handle(x)):
            return self.custom.all_reduce(x)
        if self._via_host(x):
            h = x.float().cpu()
            dist.all_reduce(h, group=self.group)
            x.copy_(h)
            return x
        dist.all_reduce(x, group=self.group)
        return x

    def fused_norm_ok(self, rows: int, hidden: int, device_type: str = "cuda") -> bool:
        """Can residual-add + RMSNorm ride in the all-reduce (custom collectives on)?"""
        return (self.world_size > 1 and device_type == "cuda" and self._custom_on()
                and self.custom.can_fuse_norm(rows, hidden))

    def fused_norm_shape(self, rows: int, hidden: int, device_type: str = "cuda") -> bool:
        """The shape rule of :meth:`fused_norm_ok` alone, whether or not the custom
        collectives are (still) up: steps of this shape keep the same projection
        kernels after a fallback to RCCL, so they produce the same bits."""
        return (self.world_size > 1 and device_type == "cuda" and hidden % 2048 == 0
                and hidden <= 8192 and rows * hidden * 2 <= self.custom_max_bytes)

    def all_reduce_add_rmsnorm(self, out, residual, weight, eps, rows, ws=None, splits=0, x=None):
        return self.custom.all_reduce_add_rmsnorm(out, residual, weight, eps, rows, ws=ws,
                                                  splits=splits, x=x)

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        """Concatenate rank shards along the last dim."""
        if self.world_size == 1:
            return x
        if self._custom_on() and x.is_cuda and self.custom.can_gather(x):
            return self.custom.all_gather_last(x)
        if self._via_host(x):
            h = x.cpu()
            parts = [torch.empty_like(h) for _ in range(self.world_size)]
            dist.all_gather(parts, h.contiguous(), group=self.group)
            return torch.cat(parts, dim=-1).to(x.device)
        parts = [torch.empty_like(x) for _ in range(self.world_size)]
        dist.all_gather(parts, x.contiguous(), group=self.group)
        return torch.cat(parts, dim=-1)

    # ---------------------------------------------------------------- fault contract
    @property
    def error_flag(self) -> Optional[torch.Tensor]:
        """Device int32 flag the custom collectives' timeouts land in (None when the
        custom path is off): the runner copies it to the host with each step's
        sampled ids and fails the step when it is set."""
        return self.custom.err_flag if self._custom_on() else None

    def export_error(self):
        if self._custom_on():
            self.custom.export_error()

    def disable_custom(self, reason: str = ""):
        if self.custom is not None:
            self.custom.disable(reason)

    def graph_safe(self) -> bool:
        """Can this group's collectives be captured in a hipGraph?"""
        if self.world_size == 1:
            return True
        if self._host_staged is None:
            self._host_staged = dist.get_backend(self.group) != "nccl"
        return not self._host_staged or self._custom_on()

    def min_int(self, v: int) -> int:
        """Smallest value of ``v`` over the group (e.g. KV blocks every rank can hold)."""
        if self.world_size == 1:
            return int(v)
        dev = "cuda" if dist.get_backend(self.group) == "nccl" else "cpu"
        t = torch.tensor([int(v)], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return int(t.item())

    def broadcast_obj(self, obj, src: int = 0):
        if self.world_size == 1:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.group)
        return lst[0]


SINGLE = TPComm()
