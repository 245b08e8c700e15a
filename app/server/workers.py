"""Data-parallel serving as N service worker processes on ONE port.

``ENGINE_DP_SIZE=N`` with ``ENGINE_DP_MODE=workers`` (the default for the native
provider): the launcher starts N worker processes.  Worker i owns GPUs
[i*tp, (i+1)*tp) and runs the whole stack -- the FastAPI ``/ws/llm`` app on the
aiohttp ASGI transport, the session / conversation managers, the voice agent and
an in-process engine.  The parent's front door (``app/server/front_door.py``,
``ENGINE_DP_FRONT=door``, the default) accepts every connection on the service port
and hands its file descriptor to the least-loaded ready worker; with
``ENGINE_DP_FRONT=reuseport`` every worker listens on the port with
``SO_REUSEPORT`` and the kernel's hash places connections instead.  A WebSocket
session lives on the worker that received it, which is also where its KV cache
(multi-turn prefix reuse) lives: session affinity comes for free.

Why not one process in front of N engine replicas (``ENGINE_DP_MODE=router``,
parallel/dp_router.py)?  Every token frame costs the service process tens of
microseconds of Python (JSON, the WebSocket write syscall, the async generator
chain); one process measured ~10k frames/s with 4 synthetic replicas at 98 % CPU
(``bench/dp_ceiling.py``, profiles/dp_ceiling_r03.log) while 8 MI355X replicas
produce ~45k tokens/s.  Workers scale the streaming side with the GPUs.

The workers still behave as ONE service (the reference runs one process,
``/root/reference/app/core/websocket_launcher.py:96-131``), through the node board
(``app/server/node_state.py``):

* ``LLM_MAX_CONNECTIONS`` caps the node, not each worker;
* a worker verifies its backend before its socket opens and exits 1 if it cannot
  (reference ``websocket_launcher.py:104-105``); the launcher exits 1 when a worker
  fails its startup check;
* ``/health`` on any worker is 503 while any worker is down, restarting or
  unhealthy; ``/stats`` sums every worker;
* the parent's monitoring port (:9092, ``main.py websocket``) reports the
  workers' request / generation / error / token counters.

The parent supervises: a worker that exits is restarted (``ENGINE_MAX_RESTARTS``
per worker); SIGTERM / SIGINT stop them all.
"""
from __future__ import annotations

import logging
import multiprocessing as mp
import os
import signal
import sys
import threading
import time
from typing import Dict, List, Optional

from app.server.front_door import DoorWorker, FrontDoor, dp_front_mode
from app.server.node_state import HEARTBEAT_S, NodeBoard

log = logging.getLogger("fasttalk.workers")

STARTUP_FAILED = 1   # exit code of a worker whose backend check failed


class _Gate:
    """ConnectionManager admission hook of worker ``index`` on the node board."""

    def __init__(self, board: NodeBoard, index: int):
        self.board, self.index = board, index

    def try_admit(self) -> bool:
        return self.board.try_admit(self.index)

    def release(self):
        self.board.release(self.index)


def _engine_snapshot(server) -> Optional[dict]:
    try:
        m = server.engine_metrics()
    except Exception:
        return None
    if not m:
        return None
    keys = ("running", "waiting", "kv_usage", "decode_steps", "decode_step_ms_avg",
            "decode_batch_avg", "prefix_cache_hit_rate", "generated_tokens")
    return {k: m[k] for k in keys if k in m and isinstance(m[k], (int, float))}


def _publisher(board: NodeBoard, index: int, server, monitor, stop: threading.Event):
    """Heartbeat + stats snapshot of this worker, every HEARTBEAT_S."""
    while not stop.is_set():
        try:
            ok = bool(server._check_backend_connection()) if server.native_handler is not None \
                else True
            board.write_snapshot(index, {
                "index": index, "pid": os.getpid(), "time": time.time(),
                "connections": server.connection_manager.get_statistics(),
                "conversations": server.conversation_manager.get_statistics(),
                "errors": server.error_handler.get_error_stats(),
                "monitor": monitor.counters(),
                "engine": _engine_snapshot(server),
            })
            board.beat(index, ok)
        except Exception as e:  # pragma: no cover - keep beating
            log.warning("worker %d: snapshot failed: %s", index, e)
        stop.wait(HEARTBEAT_S)


def worker_env(index: int, world: int, tp: int) -> Dict[str, str]:
    """Environment of DP service worker ``index``: one engine (no nested DP) whose TP
    group owns GPUs [index*tp, (index+1)*tp) (parallel/tp.py tp_device_index)."""
    return {"ENGINE_DP_SIZE": "1", "ENGINE_DEVICE_BASE": str(index * max(1, tp)),
            "FASTTALK_WORKER": f"{index}/{world}"}


def _worker_main(index: int, world: int, host: str, port: int, tp: int, board_spec=None):
    os.environ.update(worker_env(index, world, tp))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import asyncio

    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.monitoring.service_monitor import ServiceMonitor
    from app.server.asgi_aiohttp import AiohttpASGIServer
    from app.utils.config import Config

    board = NodeBoard.attach(board_spec) if board_spec else None
    cfg = Config()
    cfg.engine_dp_size = 1
    if cfg.compute_device == "cuda" and tp <= 1:
        import torch

        torch.cuda.set_device(index * tp)
        from fasttalk_llm_microservice_amd.parallel.affinity import pin_to_device

        pin_to_device(index * tp)   # this worker's threads on its GPU's NUMA-local cores
    monitor = ServiceMonitor()
    server = WebSocketLLMServer(cfg, monitor=monitor)
    monitor.attach_server(server)
    eng = getattr(server.native_handler, "engine", None) if server.native_handler else None
    inner = getattr(eng, "engine", None)
    runner = getattr(inner, "runner", None)
    if runner is not None and hasattr(runner, "warmup"):
        runner.warmup()   # decode graphs before the socket opens
    # startup verification before the port opens (reference websocket_launcher.py:104-105)
    if not server._check_backend_connection():
        log.error("DP worker %d: backend for provider '%s' is not reachable", index, cfg.llm_provider)
        if eng is not None and hasattr(eng, "shutdown"):
            eng.shutdown()
        sys.exit(STARTUP_FAILED)
    stop = threading.Event()
    if board is not None:
        server.node, server.node_index = board, index
        server.connection_manager.admission = _Gate(board, index)
        threading.Thread(target=_publisher, args=(board, index, server, monitor, stop),
                         name="fasttalk-node-publisher", daemon=True).start()
    door = board is not None and dp_front_mode() == "door"
    asgi = AiohttpASGIServer(server.app, host, port, reuse_port=not door)

    async def serve():
        door_worker = None
        if door:
            # the parent's front door accepts and hands this worker its connections
            await asgi.start(listen=False)
            door_worker = DoorWorker(asgi, board, index)
            await door_worker.start()
        else:
            await asgi.start()
        if board is not None:
            board.set(index, "ready", 1)
        log.info("DP worker %d/%d serving on %s:%d (%s)", index, world, host, port,
                 "front door" if door else "SO_REUSEPORT")
        while True:
            if door_worker is not None:
                try:
                    await asyncio.wait_for(door_worker.lost.wait(), 3600)
                except asyncio.TimeoutError:
                    continue
                # the parent is gone: nothing can reach this worker any more
                log.error("DP worker %d: front door closed; exiting", index)
                return
            await asyncio.sleep(3600)

    try:
        asyncio.run(serve())
    except (KeyboardInterrupt, SystemExit):
        pass
    finally:
        stop.set()
        if board is not None:
            board.set(index, "ready", 0)
        if eng is not None and hasattr(eng, "shutdown"):
            eng.shutdown()


class WorkerPool:
    """The parent side: starts, supervises and stops the worker processes, and owns
    the node board they share."""

    def __init__(self, world: int, host: str, port: int, tp: int = 1, max_restarts: int = 3,
                 max_connections: Optional[int] = None):
        self.world = world
        self.host = host
        self.port = port
        self.tp = max(1, tp)
        self.max_restarts = max_restarts
        if max_connections is None:
            max_connections = int(os.environ.get("LLM_MAX_CONNECTIONS", "50"))
        self.board = NodeBoard(world, max_connections)
        self.ctx = mp.get_context("spawn")
        self.procs: List[Optional[mp.Process]] = [None] * world
        self.restarts: Dict[int, int] = {i: 0 for i in range(world)}
        self._stop = False
        # ENGINE_DP_FRONT=door (default): one acceptor here places every connection on the
        # least-loaded worker; reuseport: the workers share the port (kernel hash)
        self.front_mode = dp_front_mode()
        self.door: Optional[FrontDoor] = None

    def _spawn(self, i: int):
        p = self.ctx.Process(target=_worker_main,
                             args=(i, self.world, self.host, self.port, self.tp, self.board.spec()),
                             name=f"fasttalk-worker{i}", daemon=False)
        p.start()
        self.procs[i] = p
        self.board.worker_started(i, p.pid, self.restarts[i])

    def start(self) -> "WorkerPool":
        if self.front_mode == "door":
            self.door = FrontDoor(self.board, self.host, self.port).start()
        for i in range(self.world):
            self._spawn(i)
        return self

    def wait_ready(self, timeout: float = 1800.0, poll_s: float = 0.2) -> bool:
        """Blocks until every worker serves.  False when one exits first (with its
        startup-check code or otherwise) or the timeout passes."""
        t_end = time.time() + timeout
        while time.time() < t_end:
            ws = self.board.workers()
            if all(w["ready"] for w in ws):
                return True
            for i, p in enumerate(self.procs):
                if p is not None and not p.is_alive():
                    log.error("DP worker %d exited during startup (code %s)", i, p.exitcode)
                    return False
            time.sleep(poll_s)
        return False

    def alive(self) -> List[bool]:
        return [p is not None and p.is_alive() for p in self.procs]

    def supervise_once(self):
        for i, p in enumerate(self.procs):
            if self._stop or p is None or p.is_alive():
                continue
            self.board.worker_gone(i)
            if self.restarts[i] >= self.max_restarts:
                log.error("DP worker %d exited (code %s); restart budget spent", i, p.exitcode)
                self.procs[i] = None
                continue
            self.restarts[i] += 1
            log.error("DP worker %d exited (code %s); restarting (%d/%d)", i, p.exitcode,
                      self.restarts[i], self.max_restarts)
            self._spawn(i)

    def run(self, poll_s: float = 0.5):
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
        for i in range(self.world):
            self.board.worker_gone(i)
        if self.door is not None:
            self.door.stop()
            self.door = None

    def close(self):
        self.board.close()
