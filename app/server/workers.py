"""Data-parallel serving as N service worker processes on ONE port.

``ENGINE_DP_SIZE=N`` with ``ENGINE_DP_MODE=workers`` (the default for the native
provider): the launcher starts N worker processes.  Worker i owns GPUs
[i*tp, (i+1)*tp) and runs the whole stack -- the FastAPI ``/ws/llm`` app on the
aiohttp ASGI transport, the session / conversation managers, the voice agent and
an in-process engine -- and every worker listens on the service port with
``SO_REUSEPORT``, so the kernel spreads incoming connections over them.  A
WebSocket session lives on the worker that accepted it, which is also where its
KV cache (multi-turn prefix reuse) lives: session affinity comes for free.

Why not one process in front of N engine replicas (``ENGINE_DP_MODE=router``,
parallel/dp_router.py)?  Every token frame costs the service process tens of
microseconds of Python (JSON, the WebSocket write syscall, the async generator
chain); one process measured ~10k frames/s with 4 synthetic replicas at 98 % CPU
(``bench/dp_ceiling.py``, profiles/dp_ceiling_r03.log) while 8 MI355X replicas
produce ~45k tokens/s.  Workers scale the streaming side with the GPUs.

The parent supervises: a worker that exits is restarted (``ENGINE_MAX_RESTARTS``
per worker); SIGTERM / SIGINT stop them all.  Each worker's ``/health`` and
``/stats`` describe that worker (the reference serves one process as well,
``/root/reference/app/core/websocket_launcher.py:122-128``); the monitoring port
stays in the parent.
"""
from __future__ import annotations

import logging
import multiprocessing as mp
import os
import signal
import sys
import time
from typing import Dict, List, Optional

log = logging.getLogger("fasttalk.workers")


def _worker_main(index: int, world: int, host: str, port: int, tp: int):
    os.environ["ENGINE_DP_SIZE"] = "1"
    os.environ["ENGINE_DEVICE_BASE"] = str(index * tp)
    os.environ["FASTTALK_WORKER"] = f"{index}/{world}"
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import asyncio

    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.server.asgi_aiohttp import AiohttpASGIServer
    from app.utils.config import Config

    cfg = Config()
    cfg.engine_dp_size = 1
    if cfg.compute_device == "cuda" and tp <= 1:
        import torch

        torch.cuda.set_device(index * tp)
    server = WebSocketLLMServer(cfg)
    eng = getattr(server.native_handler, "engine", None) if server.native_handler else None
    inner = getattr(eng, "engine", None)
    runner = getattr(inner, "runner", None)
    if runner is not None and hasattr(runner, "warmup"):
        runner.warmup()   # decode graphs before the socket opens
    asgi = AiohttpASGIServer(server.app, host, port, reuse_port=True)
    log.info("DP worker %d/%d serving on %s:%d", index, world, host, port)
    try:
        asyncio.run(asgi.serve_forever())
    except (KeyboardInterrupt, SystemExit):
        pass
    finally:
        if eng is not None and hasattr(eng, "shutdown"):
            eng.shutdown()


class WorkerPool:
    """The parent side: starts, supervises and stops the worker processes."""

    def __init__(self, world: int, host: str, port: int, tp: int = 1, max_restarts: int = 3):
        self.world = world
        self.host = host
        self.port = port
        self.tp = max(1, tp)
        self.max_restarts = max_restarts
        self.ctx = mp.get_context("spawn")
        self.procs: List[Optional[mp.Process]] = [None] * world
        self.restarts: Dict[int, int] = {i: 0 for i in range(world)}
        self._stop = False

    def _spawn(self, i: int):
        p = self.ctx.Process(target=_worker_main, args=(i, self.world, self.host, self.port, self.tp),
                             name=f"fasttalk-worker{i}", daemon=False)
        p.start()
        self.procs[i] = p

    def start(self) -> "WorkerPool":
        for i in range(self.world):
            self._spawn(i)
        return self

    def alive(self) -> List[bool]:
        return [p is not None and p.is_alive() for p in self.procs]

    def supervise_once(self):
        for i, p in enumerate(self.procs):
            if self._stop or p is None or p.is_alive():
                continue
            if self.restarts[i] >= self.max_restarts:
                log.error("DP worker %d exited (code %s); restart budget spent", i, p.exitcode)
                self.procs[i] = None
                continue
            self.restarts[i] += 1
            log.error("DP worker %d exited (code %s); restarting (%d/%d)", i, p.exitcode,
                      self.restarts[i], self.max_restarts)
            self._spawn(i)

    def run(self, poll_s: float = 1.0):
        """Blocks: supervises until stop() / a signal."""
        def handler(signum, frame):
            self.stop()
            sys.exit(0)

        try:
            signal.signal(signal.SIGTERM, handler)
            signal.signal(signal.SIGINT, handler)
        except ValueError:  # not the main thread
            pass
        while not self._stop:
            self.supervise_once()
            if all(p is None for p in self.procs):
                raise SystemExit("every DP worker is gone")
            time.sleep(poll_s)

    def stop(self, timeout: float = 30.0):
        self._stop = True
        for p in self.procs:
            if p is not None and p.is_alive():
                p.terminate()
        t_end = time.time() + timeout
        for p in self.procs:
            if p is not None:
                p.join(max(0.1, t_end - time.time()))
                if p.is_alive():
                    p.kill()
