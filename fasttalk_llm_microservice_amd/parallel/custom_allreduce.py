"""One-shot all-reduce over xGMI peer mappings (SURVEY.md §2.5 X1/X2, §2.7
``custom_allreduce``), for the decode-size activations tensor parallelism
reduces twice per layer.  The kernel and its signalling protocol are in
``csrc/kernels/custom_ar.hip``; this module owns the IPC plumbing:

* every rank allocates one uncached device region (``hipDeviceMallocUncached``:
  epoch/error/arrival words, 8 signal slots, 2 staging buffers of
  ``max_bytes``) and exports it with ``hipIpcGetMemHandle``;
* the handles are exchanged once with ``all_gather_object`` over the TP group
  and opened with ``hipIpcOpenMemHandle``; the W base pointers live in a device
  int64 tensor, so the all-reduce is one kernel with fixed arguments and can be
  captured in the decode hipGraph;
* a wait that runs past the spin budget sets an error word instead of hanging
  the GPU; :meth:`healthy` reads it and the communicator then falls back to RCCL.

Opt-in (``ENGINE_CUSTOM_ALLREDUCE=1``): messages above ``max_bytes`` (prefill)
always go through RCCL.
"""
from __future__ import annotations

import logging
from typing import List, Optional

import torch
import torch.distributed as dist

log = logging.getLogger("fasttalk.custom_ar")


class CustomAllReduce:
    SUPPORTED_WORLD = (2, 4, 8)

    def __init__(self, group, rank: int, world: int, device: torch.device,
                 max_bytes: int = 8 << 20, spin_budget: int = 1 << 26):
        from .. import ops

        if world not in self.SUPPORTED_WORLD:
            raise ValueError(f"custom all-reduce supports world sizes {self.SUPPORTED_WORLD}")
        self._C = ops.native()
        self.rank, self.world = rank, world
        self.max_bytes = int(max_bytes)
        self.spin_budget = int(spin_budget)
        size = int(self._C.custom_ar_header_bytes()) + 2 * self.max_bytes
        self.base = int(self._C.custom_ar_alloc(size))
        handle = self._C.custom_ar_handle(self.base)
        handles: List[Optional[bytes]] = [None] * world
        dist.all_gather_object(handles, handle, group=group)
        self._opened: List[int] = []
        ptrs = []
        for r, h in enumerate(handles):
            if r == rank:
                ptrs.append(self.base)
            else:
                p = int(self._C.custom_ar_open(h))
                self._opened.append(p)
                ptrs.append(p)
        self.peers = torch.tensor(ptrs, dtype=torch.int64, device=device)
        self.failed = False
        log.info("custom all-reduce ready: rank %d/%d, %d MiB staging", rank, world,
                 self.max_bytes >> 20)

    def can_handle(self, x: torch.Tensor) -> bool:
        return (not self.failed and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % 8 == 0 and x.numel() * 2 <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        self._C.custom_ar_allreduce(x, x, self.peers, self.rank, self.world, self.max_bytes,
                                    self.spin_budget)
        return x

    def healthy(self) -> bool:
        """Synchronising check of the error word (call outside hot loops)."""
        if not self.failed and int(self._C.custom_ar_error(self.base)):
            log.error("custom all-reduce timed out waiting for a peer; falling back to RCCL")
            self.failed = True
        return not self.failed

    def close(self):
        for p in self._opened:
            try:
                self._C.custom_ar_close(p)
            except Exception:
                pass
        self._opened = []
        if self.base:
            try:
                self._C.custom_ar_free(self.base)
            except Exception:
                pass
            self.base = 0
