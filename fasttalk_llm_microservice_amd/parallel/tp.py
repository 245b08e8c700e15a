"""Tensor parallelism: one process per GPU, RCCL over xGMI (SURVEY.md §2.6 P1,
§2.7; BASELINE config 4 "Llama-3-70B TP=8").

Rank 0 owns everything stateful -- scheduler, KV block manager, detokenizer,
service -- and its :class:`~..engine.runner.ModelRunner` broadcasts each
step's host inputs through :class:`.shm_broadcast.ShmBroadcast`.  Ranks 1..N-1
are *workers*: the same ``ModelRunner`` on their GPU with 1/N of every weight
(column-parallel QKV / gate_up, row-parallel O / down, vocab-parallel LM
head), replaying the identical kernel + collective sequence (the same decode
hipGraph buckets, captured in lock-step) for every message.  Per layer the
only cross-GPU traffic is two all-reduces of the [tokens, hidden] activations
plus one all-gather of the logits per step (§2.5 X1/X2/X4).

Two launch modes:

* ``spawn_tp_engine(cfg)`` -- the service process becomes rank 0 and starts the
  workers itself (``multiprocessing`` spawn, rendezvous on 127.0.0.1).
* ``torchrun_tp(cfg)`` -- all ranks were started by ``torch.distributed.run``;
  rank 0 gets an engine, the others enter :func:`worker_loop` and return when
  rank 0 shuts down.
"""
from __future__ import annotations

import logging
import multiprocessing as mp
import os
import socket
import threading
import time
from typing import List, Optional

import torch
import torch.distributed as dist

from .comm import TPComm
from .shm_broadcast import ShmBroadcast

log = logging.getLogger("fasttalk.tp")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _backend(device: str, cfg=None) -> str:
    """RCCL on GPUs.  ``tp_share_device`` (tests: every rank on ONE GPU, which RCCL
    refuses) runs control over gloo and the data path over the custom xGMI/IPC
    collectives, with gloo host staging as the fallback."""
    if device == "cuda" and not (cfg is not None and cfg.tp_share_device):
        return "nccl"
    return "gloo"


def _set_device(device: str, index: int):
    if device == "cuda":
        torch.cuda.set_device(index)


def _exit_with_parent(what: str):
    """Workers die with the rank-0 process that spawned them even when they are
    stuck inside a collective that will never complete (the step loop cannot
    notice then): a daemon thread polls the parent pid once a second."""
    ppid = os.getppid()

    def watch():
        while True:
            time.sleep(1.0)
            if os.getppid() != ppid:
                log.error("%s: rank 0 (pid %d) is gone; exiting", what, ppid)
                os._exit(3)

    threading.Thread(target=watch, name="fasttalk-tp-parent-watch", daemon=True).start()


def _maybe_custom_ar(cfg, comm: TPComm, device: str):
    """Every rank of the group calls this at the same point (it is collective)."""
    if not (getattr(cfg, "custom_allreduce", False) and device == "cuda"):
        return
    from .custom_allreduce import CustomAllReduce

    if comm.world_size not in CustomAllReduce.SUPPORTED_WORLD:
        return
    ar, ok = None, 1
    try:
        # ranks sharing ONE device (tests / rehearsals): W-1 collectives spin on the same
        # CUs the last rank computes on -- cap their grids at 16 workgroups
        ar = CustomAllReduce(comm.group, comm.rank, comm.world_size,
                             torch.device("cuda", torch.cuda.current_device()),
                             max_blocks=16 if getattr(cfg, "tp_share_device", False) else None,
                             shared_device=bool(getattr(cfg, "tp_share_device", False)))
    except Exception as e:  # e.g. IPC mapping refused: the group stays on RCCL
        log.warning("custom all-reduce unavailable on rank %d: %s", comm.rank, e)
        ok = 0
    if comm.min_int(ok):    # every rank mapped every peer
        comm.custom = ar
    elif ar is not None:
        ar.close()


def _make_runner(cfg, comm: TPComm):
    from ..engine.runner import ModelRunner
    from ..models.config import resolve_model

    mcfg = resolve_model(cfg.weights if cfg.weights not in ("random", None, "") else cfg.model)
    return ModelRunner(cfg, mcfg, comm)


def worker_loop(cfg, comm: TPComm, bcast: ShmBroadcast):
    """Runs broadcast steps until rank 0 sends ``stop``."""
    runner = _make_runner(cfg, comm)
    log.info("TP worker %d/%d ready on %s", comm.rank, comm.world_size, runner.device)
    try:
        while runner.run_remote(bcast.recv()):
            pass
    finally:
        bcast.close()


def tp_device_index(device_base: int, rank: int, share_device: bool = False) -> int:
    """GPU of TP rank ``rank`` in a group whose first GPU is ``device_base`` (a DP
    service worker i with TP size t owns GPUs [i*t, (i+1)*t): app/server/workers.py).
    ``share_device``: every rank on ``device_base`` (tests / rehearsals)."""
    return int(device_base) + (0 if share_device else int(rank))


def _spawned_worker(rank: int, world: int, port: int, bcast_name: str, cfg, device: str,
                    device_base: int):
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    _exit_with_parent(f"TP worker {rank}")
    dev_index = tp_device_index(device_base, rank, cfg.tp_share_device)
    _set_device(device, dev_index)
    if device == "cuda" and not cfg.tp_share_device:
        from .affinity import pin_to_device

        pin_to_device(dev_index)   # each TP rank on its own GPU's NUMA-local cores
    kw = {}
    if device == "cuda" and not cfg.tp_share_device:
        kw["device_id"] = torch.device(f"cuda:{dev_index}")
    dist.init_process_group(_backend(device, cfg), init_method=f"tcp://127.0.0.1:{port}",
                            rank=rank, world_size=world, **kw)
    comm = TPComm(dist.group.WORLD, rank, world)
    _maybe_custom_ar(cfg, comm, device)
    bcast = ShmBroadcast(world - 1, name=bcast_name, create=False, reader_index=rank - 1)
    try:
        worker_loop(cfg, comm, bcast)
    finally:
        dist.destroy_process_group()


class TPGroup:
    """Rank-0 side of a spawned TP group: owns the worker processes, the process
    group and the broadcast ring."""

    def __init__(self, cfg, device_base: int = 0):
        self.cfg = cfg
        self.world = cfg.tp_size
        self.device = cfg.resolved_device()
        self.device_base = device_base
        self.port = _free_port()
        self.bcast = ShmBroadcast(self.world - 1)
        self.bcast.liveness = self.alive
        ctx = mp.get_context("spawn")
        self.procs: List[mp.Process] = []
        for r in range(1, self.world):
            p = ctx.Process(target=_spawned_worker, name=f"fasttalk-tp{r}", daemon=True,
                            args=(r, self.world, self.port, self.bcast.name, cfg, self.device,
                                  device_base))
            p.start()
            self.procs.append(p)
        dev0 = tp_device_index(device_base, 0, cfg.tp_share_device)
        _set_device(self.device, dev0)
        kw = {}
        if self.device == "cuda" and not cfg.tp_share_device:
            kw["device_id"] = torch.device(f"cuda:{dev0}")
        dist.init_process_group(_backend(self.device, cfg),
                                init_method=f"tcp://127.0.0.1:{self.port}",
                                rank=0, world_size=self.world, **kw)
        self.comm = TPComm(dist.group.WORLD, 0, self.world)
        _maybe_custom_ar(cfg, self.comm, self.device)

    def attach(self, runner):
        runner.bcast = self.bcast

    def shutdown(self):
        if self.bcast is None:
            return
        try:
            self.bcast.send(("stop", None, None), timeout=30)
        except Exception:
            pass
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        self.bcast.close()
        self.bcast = None
        if dist.is_initialized():
            dist.destroy_process_group()

    def alive(self) -> bool:
        """Every worker process still running (wired into the engine's health)."""
        return all(p.is_alive() for p in self.procs)


def spawn_tp_engine(cfg, device_base: int = 0):
    """Returns an :class:`~..engine.engine.LLMEngine` that is rank 0 of a freshly
    spawned TP group (``engine.tp_group`` keeps the group for shutdown)."""
    from ..engine.engine import LLMEngine

    group = TPGroup(cfg, device_base)
    try:
        runner = _make_runner(cfg, group.comm)
        group.attach(runner)
        eng = LLMEngine(cfg, comm=group.comm, runner=runner)
    except BaseException:
        group.shutdown()
        raise
    eng.tp_group = group
    return eng


def torchrun_tp(cfg) -> Optional[object]:
    """Under ``torch.distributed.run``: rank 0 returns an LLMEngine (rank 0 of
    the TP group spanning the whole job), other ranks serve as workers and
    return None once rank 0 stops them."""
    from ..engine.engine import LLMEngine

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = cfg.resolved_device()
    dev_index = 0 if cfg.tp_share_device else local
    _set_device(device, dev_index)
    if not dist.is_initialized():
        kw = {"device_id": torch.device(f"cuda:{dev_index}")} \
            if device == "cuda" and not cfg.tp_share_device else {}
        dist.init_process_group(_backend(device, cfg), **kw)
    comm = TPComm(dist.group.WORLD, rank, world)
    _maybe_custom_ar(cfg, comm, device)
    name = [None]
    bcast = None
    if rank == 0:
        bcast = ShmBroadcast(world - 1)
        name[0] = bcast.name
    dist.broadcast_object_list(name, src=0)
    if rank != 0:
        bcast = ShmBroadcast(world - 1, name=name[0], create=False, reader_index=rank - 1)
        worker_loop(cfg, comm, bcast)
        return None
    runner = _make_runner(cfg, comm)
    runner.bcast = bcast

    class _Group:
        def shutdown(self):
            bcast.send(("stop", None, None), timeout=30)
            bcast.close()

    eng = LLMEngine(cfg, comm=comm, runner=runner)
    eng.tp_group = _Group()
    return eng
