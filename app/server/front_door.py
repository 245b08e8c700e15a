"""The DP front door: ONE acceptor places every new connection on the least-loaded
service worker (``ENGINE_DP_FRONT=door``, the default for ``ENGINE_DP_SIZE`` > 1).

The reference is one process that sees every session and enforces one cap
(``/root/reference/app/core/websocket_launcher.py:122-128``,
``/root/reference/app/utils/connection_manager.py:128-133``).  With N worker
processes (``app/server/workers.py``, one engine / GPU each) the question is which
worker a new WebSocket session lands on -- its KV cache, its conversation history
and its share of the GPU follow it for the whole session.  ``SO_REUSEPORT`` leaves
that to the kernel's 4-tuple hash: no balance (4 sessions over 2 workers all landed
on one in 2 of 3 runs; 400 sessions over 8 GPUs spread binomially, the busiest GPU
carrying ~65 while another carries ~35).

The door instead:

* listens on the service port in the parent (the WorkerPool process, or rank 0 of
  ``bench.py``), accepts each TCP connection, and passes its file descriptor over a
  ``SOCK_SEQPACKET`` unix socket (``SCM_RIGHTS``) to the live, ready worker with
  the fewest open connections -- the worker's own count on the node board
  (``conns``) plus the hand-offs it has not received yet (``sent - recv``), so a
  burst of connects is spread before any worker has reported back; ties rotate;
* never proxies a byte: the worker owns the socket from then on (aiohttp
  ``connect_accepted_socket``), so a session stays on its worker (affinity) and the
  parent costs one ``accept`` + one ``sendmsg`` per connection;
* opens the port only once a worker has registered (a service whose workers all
  fail their startup check never listens, as before), answers ``503`` when no
  worker is live, and routes around a worker that died (its control socket breaks).

Worker side: :class:`DoorWorker` registers on the control socket once its engine is
warm, adopts every descriptor it is handed, and keeps its ``conns`` / ``recv``
counters on the board current.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import socket
import threading
import time
from typing import Dict, List, Optional

from app.server.node_state import NodeBoard

log = logging.getLogger("fasttalk.front_door")

CTL_NAME = "front.sock"


def dp_front_mode() -> str:
    """``door`` (default): one acceptor, least-loaded placement; ``reuseport``: every
    worker listens on the port with SO_REUSEPORT (kernel hash placement)."""
    m = os.environ.get("ENGINE_DP_FRONT", "door").strip().lower()
    return m if m in ("door", "reuseport") else "door"


def _refuse(conn: socket.socket, reason: str):
    body = json.dumps({"status": "unavailable", "error": reason}).encode()
    try:
        conn.settimeout(1.0)
        conn.sendall(b"HTTP/1.1 503 Service Unavailable\r\nContent-Type: application/json\r\n"
                     b"Content-Length: " + str(len(body)).encode() + b"\r\nConnection: close\r\n\r\n" + body)
    except OSError:
        pass
    finally:
        conn.close()


class FrontDoor:
    """Parent side: the listening socket and the per-worker control sockets."""

    def __init__(self, board: NodeBoard, host: str, port: int, backlog: int = 4096):
        self.board = board
        self.host, self.port = host, int(port)
        self.backlog = int(backlog)
        self.world = board.world
        self.ctl_path = os.path.join(board.path, CTL_NAME)
        self._ctl: Dict[int, socket.socket] = {}
        self._sent: List[int] = [0] * self.world
        self._lock = threading.Lock()
        self._registered = threading.Event()
        self.listening = threading.Event()
        self._stop = threading.Event()
        self._rr = 0
        self._srv: Optional[socket.socket] = None
        self._ctl_srv: Optional[socket.socket] = None
        self._threads: List[threading.Thread] = []
        self.stats = {"handed": 0, "refused": 0, "rerouted": 0, "per_worker": [0] * self.world}

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "FrontDoor":
        try:
            os.unlink(self.ctl_path)
        except FileNotFoundError:
            pass
        s = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
        s.bind(self.ctl_path)
        s.listen(max(64, 4 * self.world))
        s.settimeout(0.25)
        self._ctl_srv = s
        for target, name in ((self._ctl_loop, "fasttalk-door-ctl"), (self._accept_loop, "fasttalk-door")):
            t = threading.Thread(target=target, name=name, daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)
        for s in [self._srv, self._ctl_srv] + list(self._ctl.values()):
            if s is not None:
                try:
                    s.close()
                except OSError:
                    pass
        self._ctl.clear()
        try:
            os.unlink(self.ctl_path)
        except OSError:
            pass

    # ------------------------------------------------------------------ control socket
    def _ctl_loop(self):
        while not self._stop.is_set():
            try:
                c, _ = self._ctl_srv.accept()
            except socket.timeout:
                continue
            except OSError:
                return
            try:
                c.settimeout(10.0)
                msg = c.recv(64)
                c.settimeout(None)
                if not msg.startswith(b"W"):
                    raise ValueError(msg)
                index = int(msg[1:].decode().strip())
                if not 0 <= index < self.world:
                    raise ValueError(index)
            except (OSError, ValueError) as e:
                log.warning("front door: bad worker registration: %s", e)
                c.close()
                continue
            with self._lock:
                old = self._ctl.pop(index, None)
                if old is not None:
                    old.close()
                self._ctl[index] = c
                # a (re)started worker reports recv from 0: nothing is in flight to it
                self._sent[index] = int(self.board.get(index, "recv"))
            log.info("front door: worker %d registered", index)
            self._registered.set()

    # ------------------------------------------------------------------ placement
    def load(self, index: int) -> float:
        """Open connections of worker ``index`` plus hand-offs it has not received."""
        pending = max(0.0, self._sent[index] - self.board.get(index, "recv"))
        return self.board.get(index, "conns") + pending

    def pick(self, exclude=()) -> Optional[int]:
        ws = self.board.workers()
        best, best_load = None, 0.0
        for k in range(self.world):
            i = (self._rr + k) % self.world
            if i in exclude or i not in self._ctl:
                continue
            w = ws[i]
            # a worker whose event loop stopped beating (alive but stalled) gets no new
            # sessions: it would not read its control socket either
            if not (w["alive"] and w["ready"] and w["heartbeat_fresh"]):
                continue
            ld = self.load(i)
            if best is None or ld < best_load:
                best, best_load = i, ld
        self._rr = (self._rr + 1) % self.world
        return best

    def _hand(self, conn: socket.socket):
        tried = set()
        while True:
            with self._lock:
                i = self.pick(tried)
                if i is None:
                    self.stats["refused"] += 1
                    break
                ctl = self._ctl[i]
                try:
                    # never block the accept thread (and, under the lock, every other
                    # placement) on one worker whose socket buffer is full: MSG_DONTWAIT,
                    # and a full buffer (EAGAIN) reroutes like an unreachable worker
                    socket.send_fds(ctl, [b"c"], [conn.fileno()], socket.MSG_DONTWAIT)
                except BlockingIOError:
                    log.warning("front door: worker %d not reading its hand-offs; rerouting", i)
                    tried.add(i)
                    self.stats["rerouted"] += 1
                    continue
                except OSError as e:
                    log.warning("front door: worker %d unreachable (%s); rerouting", i, e)
                    self._ctl.pop(i, None)
                    ctl.close()
                    tried.add(i)
                    self.stats["rerouted"] += 1
                    continue
                self._sent[i] += 1
                self.stats["handed"] += 1
                self.stats["per_worker"][i] += 1
            conn.close()   # the worker holds its own duplicate now
            return
        _refuse(conn, "no service worker is ready")

    def _accept_loop(self):
        while not self._registered.wait(0.25):
            if self._stop.is_set():
                return
        try:
            srv = socket.create_server((self.host, self.port), backlog=self.backlog, reuse_port=False)
        except OSError as e:
            log.error("front door: cannot listen on %s:%d: %s", self.host, self.port, e)
            return
        srv.settimeout(0.25)
        self._srv = srv
        self.port = srv.getsockname()[1]
        self.listening.set()
        log.info("front door listening on %s:%d for %d workers", self.host, self.port, self.world)
        while not self._stop.is_set():
            try:
                conn, _ = srv.accept()
            except socket.timeout:
                continue
            except OSError:
                if self._stop.is_set():
                    return
                time.sleep(0.01)
                continue
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self._hand(conn)


class DoorWorker:
    """Worker side: adopt connections handed over by the front door into this
    worker's aiohttp server (``AiohttpASGIServer.start(listen=False)``)."""

    def __init__(self, asgi, board: NodeBoard, index: int, ctl_path: Optional[str] = None):
        self.asgi = asgi
        self.board = board
        self.index = index
        self.ctl_path = ctl_path or os.path.join(board.path, CTL_NAME)
        self.sock: Optional[socket.socket] = None
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.lost = asyncio.Event()
        self.adopted = 0

    async def start(self, timeout: float = 30.0):
        self.loop = asyncio.get_running_loop()
        srv = self.asgi.protocol_factory()
        orig_lost = srv.connection_lost
        board, index = self.board, self.index

        def connection_lost(handler, exc=None):
            board.add(index, "conns", -1)
            orig_lost(handler, exc)

        srv.connection_lost = connection_lost   # count this worker's open sockets
        s = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
        t_end = time.time() + timeout
        while True:
            try:
                s.connect(self.ctl_path)
                break
            except (FileNotFoundError, ConnectionRefusedError):
                if time.time() > t_end:
                    raise
                await asyncio.sleep(0.1)
        s.sendall(f"W{self.index}\n".encode())
        s.setblocking(False)
        self.sock = s
        self.loop.add_reader(s.fileno(), self._on_ctl)

    def _on_ctl(self):
        while True:
            try:
                msg, fds, _flags, _addr = socket.recv_fds(self.sock, 16, 4)
            except BlockingIOError:
                return
            except OSError:
                msg, fds = b"", []
            if not msg and not fds:   # the door went away
                self.loop.remove_reader(self.sock.fileno())
                self.lost.set()
                return
            for fd in fds:
                conn = socket.socket(fileno=fd)
                conn.setblocking(False)
                self.board.add(self.index, "conns", 1)
                self.board.add(self.index, "recv", 1)
                self.adopted += 1
                self.loop.create_task(self._adopt(conn))

    async def _adopt(self, conn: socket.socket):
        try:
            await self.loop.connect_accepted_socket(self.asgi.protocol_factory(), sock=conn)
        except Exception as e:   # peer already gone: nothing was counted by the server
            log.debug("front door: adopt failed: %s", e)
            self.board.add(self.index, "conns", -1)
            conn.close()

    def close(self):
        if self.sock is not None:
            try:
                if self.loop is not None:
                    self.loop.remove_reader(self.sock.fileno())
            except (ValueError, OSError, RuntimeError):
                pass
            self.sock.close()
            self.sock = None
