"""All-reduce / all-gather over xGMI peer mappings (SURVEY.md §2.5 X1/X2/X4,
§2.7 ``custom_allreduce``), for the decode-size activations tensor parallelism
reduces twice per layer and the vocab-sharded logits it gathers once per step.
The kernels and their signalling protocol are in ``csrc/kernels/custom_ar.hip``;
this module owns the IPC plumbing and the fault contract:

* every rank allocates one uncached device region (``hipDeviceMallocUncached``:
  epoch/error/arrival words, 8 signal slots, 2 staging buffers of
  ``max_bytes``) and exports it with ``hipIpcGetMemHandle``;
* the handles are exchanged once with ``all_gather_object`` over the TP group
  and opened with ``hipIpcOpenMemHandle``; the W base pointers live in a device
  int64 tensor, so the all-reduce is one kernel with fixed arguments and can be
  captured in the decode hipGraph;
* one-shot (every rank reads all W inputs) below ``two_shot_bytes``, two-shot
  (reduce-scatter + all-gather, 2(W-1)/W of the remote bytes, one more
  barrier) above it.  W=2 is always one-shot (both move n remote bytes).  The
  default crossover (512 KiB at W=8, 1 MiB at W=4; ``ENGINE_CUSTOM_AR_TWO_SHOT``)
  comes from the link model -- 7 xGMI links per GPU, a few microseconds per
  cross-rank barrier -- not from a measurement: no multi-GPU box was available;
* a wait that runs past the spin budget sets a sticky error word instead of
  hanging the GPU, and the kernel returns with ``out`` NOT reduced.  Every
  later collective on that rank returns at once.  :meth:`export_error` (in
  every decode graph and after every eager step) folds all W error words into
  :attr:`err_flag`, which the runner copies to the host with the sampled ids:
  a set flag fails the step -- its tokens are discarded, never emitted -- and
  the whole group switches to RCCL (:meth:`disable` on every rank, graphs
  recaptured).

On by default for tensor parallelism on GPUs (``ENGINE_CUSTOM_ALLREDUCE=0`` turns it
off, engine/config.py); messages above ``max_bytes`` (long prefills) always go
through RCCL.
"""
from __future__ import annotations

import contextlib
import logging
import os
from typing import List, Optional

import torch
import torch.distributed as dist

log = logging.getLogger("fasttalk.custom_ar")


class CustomAllReduce:
    SUPPORTED_WORLD = (2, 4, 8)

    def __init__(self, group, rank: int, world: int, device: torch.device,
                 max_bytes: int = 8 << 20, spin_budget: Optional[int] = None,
                 two_shot_bytes: Optional[int] = None, max_blocks: Optional[int] = None,
                 shared_device: bool = False):
        from .. import ops

        if world not in self.SUPPORTED_WORLD:
            raise ValueError(f"custom all-reduce supports world sizes {self.SUPPORTED_WORLD}")
        self._C = ops.native()
        self.rank, self.world = rank, world
        # grid cap of the collectives: ranks that share one device keep it small, so the
        # kernels spinning for a late peer leave that peer CUs to compute on
        if max_blocks is None:
            max_blocks = int(os.environ.get("ENGINE_CUSTOM_AR_BLOCKS", "128"))
        self.max_blocks = int(max_blocks)
        self._C.custom_ar_set_max_blocks(self.max_blocks)
        self.max_bytes = int(max_bytes)
        # spin budgets: ~0.19 us per spin on a GPU of its own.  A timeout raises
        # CommFault and drops the group to RCCL for the rest of the process, so the budget
        # must cover real host / scheduling stalls of a peer, and no multi-GPU run has
        # measured those yet (no 8-GPU node in this environment): every group keeps the
        # conservative 2^25 spins (~6-12 s) and 2^28 for its first steps (lazy library /
        # code-object loads, allocator growth on one rank while the others already wait).
        # ENGINE_CUSTOM_AR_SPIN / _SPIN_FIRST tune them once a multi-GPU run has
        # measured the stalls.
        self.shared_device = bool(shared_device)
        default_spin, default_first = 1 << 25, 1 << 28
        if spin_budget is None:
            spin_budget = int(os.environ.get("ENGINE_CUSTOM_AR_SPIN", str(default_spin)))
        self.spin_budget = int(spin_budget)
        self.first_spin_budget = max(self.spin_budget,
                                     int(os.environ.get("ENGINE_CUSTOM_AR_SPIN_FIRST",
                                                        str(default_first))))
        if two_shot_bytes is None:
            env = os.environ.get("ENGINE_CUSTOM_AR_TWO_SHOT")
            two_shot_bytes = int(env) if env else {8: 512 << 10, 4: 1 << 20}.get(world, 1 << 62)
        self.two_shot_bytes = int(two_shot_bytes)
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
        self.err_flag = torch.zeros(1, dtype=torch.int32, device=device)
        self.failed = False
        log.info("custom all-reduce ready: rank %d/%d, %d MiB staging", rank, world,
                 self.max_bytes >> 20)

    def can_handle(self, x: torch.Tensor) -> bool:
        return (not self.failed and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % 8 == 0 and x.numel() * 2 <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        two = x.numel() * 2 >= self.two_shot_bytes
        self._C.custom_ar_allreduce(x, x, self.peers, self.rank, self.world, self.max_bytes,
                                    self.spin_budget, two)
        return x

    def can_fuse_norm(self, rows: int, hidden: int) -> bool:
        return (not self.failed and hidden % 2048 == 0 and hidden <= 8192
                and rows * hidden * 2 <= self.max_bytes)

    def all_reduce_add_rmsnorm(self, out: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor,
                               eps: float, rows: int, ws: Optional[torch.Tensor] = None,
                               splits: int = 0, x: Optional[torch.Tensor] = None) -> torch.Tensor:
        """residual[:rows] += all-reduce(partial); out = rmsnorm(residual) * weight, in
        ONE launch (the o / down epilogue of tensor parallelism).  The partial is this
        rank's split-K fp32 slabs (``ws``, ``splits``) or a bf16 block ``x``."""
        self._C.custom_ar_add_rmsnorm(out, residual, weight, float(eps), ws, int(splits), x,
                                      int(rows), self.peers, self.rank, self.world, self.max_bytes,
                                      self.spin_budget)
        return out

    def can_gather(self, x: torch.Tensor) -> bool:
        return (not self.failed and x.dtype == torch.bfloat16 and x.dim() == 2
                and x.is_contiguous() and x.shape[1] % 8 == 0
                and x.numel() * 2 <= self.max_bytes)

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        """[rows, shard] -> [rows, W * shard] in rank order."""
        out = torch.empty(x.shape[0], self.world * x.shape[1], dtype=x.dtype, device=x.device)
        self._C.custom_ar_allgather(out, x, self.peers, self.rank, self.world, self.max_bytes,
                                    self.spin_budget)
        return out

    @contextlib.contextmanager
    def long_waits(self):
        """Eager collectives issued inside use the first-steps spin budget."""
        saved = self.spin_budget
        self.spin_budget = self.first_spin_budget
        try:
            yield
        finally:
            self.spin_budget = saved

    def export_error(self):
        """err_flag <- OR of every rank's error word (stream ordered, graph-safe)."""
        self._C.custom_ar_export_error(self.err_flag, self.peers, self.world)

    def disable(self, reason: str = ""):
        if not self.failed:
            log.error("custom all-reduce disabled on rank %d (%s); the group uses RCCL from now on",
                      self.rank, reason or "peer timeout")
        self.failed = True

    def peer_error(self, r: int) -> int:
        """Host read of rank r's error word through its mapping (tests, diagnostics)."""
        ptr = self.base if r == self.rank else int(self.peers[r].item())
        return int(self._C.custom_ar_error(ptr))

    def healthy(self) -> bool:
        """Synchronising check of this rank's error word (call outside hot loops)."""
        if not self.failed and int(self._C.custom_ar_error(self.base)):
            self.disable("timed out waiting for a peer")
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
