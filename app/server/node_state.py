"""Node-wide state of the DP service workers (``app/server/workers.py``), so N
worker processes behind one port behave as ONE service, as the reference's
single process does (``/root/reference/app/core/websocket_launcher.py:122-128``):

* **connection cap** -- ``LLM_MAX_CONNECTIONS`` bounds the whole node, not each
  worker (reference ``app/utils/config.py:133``,
  ``app/utils/connection_manager.py:128-133``): every admission takes an
  ``flock`` on the board, sums the live workers' open connections and counts
  itself in its worker's slot.  A lock held by a worker that dies is released
  by the kernel; the parent zeroes a dead worker's slot before respawning it;
* **health** -- the parent marks each worker alive / dead as it supervises, a
  worker marks itself ready once its engine is warm and its backend check passed,
  and beats a heartbeat; ``/health`` on any worker is 200 only when every worker
  is alive, ready, fresh and its engine healthy (503 while one is down or
  restarting);
* **stats** -- each worker publishes a JSON snapshot of its connection /
  conversation / error / monitoring counters twice a second (write + rename, no
  lock); ``/stats`` on any worker and the parent's :9092 ``/metrics`` (reference
  ``app/monitoring/service_monitor.py:125``) sum them.

The board is a small ``mmap``-ed float64 table plus the snapshot files, in one
directory under ``/dev/shm`` (tmpfs), created by the parent and removed by it.
"""
from __future__ import annotations

import contextlib
import fcntl
import json
import mmap
import os
import shutil
import tempfile
import time
from typing import Any, Dict, List, Optional

import numpy as np

# conns / recv: the front door's load signal (app/server/front_door.py) -- TCP connections
# a worker currently holds, and connections it has received from the door in total
FIELDS = ("alive", "ready", "pid", "heartbeat", "active", "restarts", "backend_ok", "started",
          "conns", "recv")
_F = {k: i for i, k in enumerate(FIELDS)}
HEARTBEAT_S = 0.5          # snapshot + heartbeat period of a worker
STALE_S = 5.0              # a worker whose heartbeat is older is reported down


class NodeBoard:
    def __init__(self, world: int, max_connections: int, path: Optional[str] = None):
        self.world = int(world)
        self.max_connections = int(max_connections)
        create = path is None
        if create:
            base = "/dev/shm" if os.path.isdir("/dev/shm") else None
            path = tempfile.mkdtemp(prefix="fasttalk-node-", dir=base)
        self.path = path
        self._owner = create
        nbytes = self.world * len(FIELDS) * 8
        fn = os.path.join(path, "board")
        if create:
            with open(fn, "wb") as f:
                f.write(b"\0" * nbytes)
            with open(os.path.join(path, "lock"), "wb"):
                pass
        self._fd = os.open(fn, os.O_RDWR)
        self._mm = mmap.mmap(self._fd, nbytes)
        self.t = np.ndarray((self.world, len(FIELDS)), dtype=np.float64, buffer=self._mm)
        self._lock_fd = os.open(os.path.join(path, "lock"), os.O_RDWR)

    def spec(self) -> Dict[str, Any]:
        """What a spawned worker needs to attach (picklable)."""
        return {"world": self.world, "max_connections": self.max_connections, "path": self.path}

    @classmethod
    def attach(cls, spec: Dict[str, Any]) -> "NodeBoard":
        return cls(spec["world"], spec["max_connections"], path=spec["path"])

    @contextlib.contextmanager
    def _locked(self):
        fcntl.flock(self._lock_fd, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(self._lock_fd, fcntl.LOCK_UN)

    # ------------------------------------------------------------------ admission
    def node_active(self) -> int:
        alive = self.t[:, _F["alive"]] > 0
        return int(self.t[alive, _F["active"]].sum())

    def try_admit(self, index: int) -> bool:
        with self._locked():
            if self.node_active() >= self.max_connections:
                return False
            self.t[index, _F["active"]] += 1
            return True

    def release(self, index: int):
        with self._locked():
            self.t[index, _F["active"]] = max(0.0, self.t[index, _F["active"]] - 1)

    # ------------------------------------------------------------------ worker side
    def set(self, index: int, field: str, value: float):
        self.t[index, _F[field]] = float(value)

    def get(self, index: int, field: str) -> float:
        return float(self.t[index, _F[field]])

    def add(self, index: int, field: str, delta: float):
        """Single-writer counter update (each worker owns its row's conns / recv)."""
        self.t[index, _F[field]] += delta

    def beat(self, index: int, backend_ok: bool):
        self.t[index, _F["backend_ok"]] = 1.0 if backend_ok else 0.0
        self.t[index, _F["heartbeat"]] = time.time()

    def write_snapshot(self, index: int, snap: Dict[str, Any]):
        fn = os.path.join(self.path, f"w{index}.json")
        tmp = fn + f".{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump(snap, f)
        os.replace(tmp, fn)

    def snapshots(self) -> List[Optional[Dict[str, Any]]]:
        out = []
        for i in range(self.world):
            try:
                with open(os.path.join(self.path, f"w{i}.json")) as f:
                    out.append(json.load(f))
            except (OSError, ValueError):
                out.append(None)
        return out

    # ------------------------------------------------------------------ parent side
    def worker_started(self, index: int, pid: int, restarts: int):
        with self._locked():
            row = self.t[index]
            row[_F["active"]] = 0
            row[_F["conns"]] = 0
            row[_F["recv"]] = 0
            row[_F["ready"]] = 0
            row[_F["backend_ok"]] = 0
            row[_F["heartbeat"]] = 0
            row[_F["pid"]] = pid
            row[_F["restarts"]] = restarts
            row[_F["started"]] = time.time()
            row[_F["alive"]] = 1

    def worker_gone(self, index: int):
        with self._locked():
            row = self.t[index]
            row[_F["alive"]] = 0
            row[_F["ready"]] = 0
            row[_F["active"]] = 0   # its sockets died with it
            row[_F["conns"]] = 0

    # ------------------------------------------------------------------ queries
    def workers(self, now: Optional[float] = None) -> List[Dict[str, Any]]:
        now = time.time() if now is None else now
        out = []
        for i in range(self.world):
            r = self.t[i]
            fresh = r[_F["heartbeat"]] > 0 and now - r[_F["heartbeat"]] < STALE_S
            out.append({"index": i, "pid": int(r[_F["pid"]]), "alive": bool(r[_F["alive"]]),
                        "ready": bool(r[_F["ready"]]), "heartbeat_fresh": bool(fresh),
                        "backend_ok": bool(r[_F["backend_ok"]]),
                        "active_connections": int(r[_F["active"]]),
                        "open_sockets": int(r[_F["conns"]]),
                        "restarts": int(r[_F["restarts"]])})
        return out

    def healthy(self) -> bool:
        return all(w["alive"] and w["ready"] and w["heartbeat_fresh"] and w["backend_ok"]
                   for w in self.workers())

    def close(self):
        try:
            self._mm.close()
        except (BufferError, ValueError):
            pass
        for fd in (self._fd, self._lock_fd):
            try:
                os.close(fd)
            except OSError:
                pass
        if self._owner:
            shutil.rmtree(self.path, ignore_errors=True)


# ---------------------------------------------------------------------- aggregation
def _sum_into(acc: Dict[str, Any], d: Dict[str, Any]):
    for k, v in d.items():
        if isinstance(v, bool) or not isinstance(v, (int, float, dict)):
            acc.setdefault(k, v)
        elif isinstance(v, dict):
            _sum_into(acc.setdefault(k, {}), v)
        else:
            acc[k] = acc.get(k, 0) + v


def merge_service_stats(parts: List[Dict[str, Any]], max_connections: int,
                        active: Optional[int] = None) -> Dict[str, Any]:
    """Sums the per-worker ``/stats`` sections (connections / conversations /
    errors) into the node view with the reference's key set.  ``active``: the live
    node-wide connection count (the board's, not the snapshots' -- those lag by up
    to one publish period)."""
    out: Dict[str, Any] = {"connections": {}, "conversations": {}, "errors": {}}
    dur_w = 0.0
    for p in parts:
        for sec in out:
            _sum_into(out[sec], p.get(sec, {}))
        c = p.get("connections", {})
        dur_w += c.get("average_session_duration_seconds", 0.0) * c.get("active_connections", 0)
    c = out["connections"]
    if active is not None:
        c["active_connections"] = active
    n = c.get("active_connections", 0)
    c["max_connections"] = max_connections
    c["utilization_percent"] = (n / max_connections * 100.0) if max_connections else 0.0
    c["average_session_duration_seconds"] = dur_w / n if n else 0.0
    # a breaker that is open on any worker is reported open for the node
    cb = {}
    for p in parts:
        for name, state in p.get("errors", {}).get("circuit_breakers", {}).items():
            if cb.get(name) in (None, "closed") or state == "open":
                cb[name] = state
    if cb:
        out["errors"]["circuit_breakers"] = cb
    return out


def merge_monitor(parts: List[Dict[str, Any]]) -> Dict[str, Any]:
    """Sums the workers' ServiceMonitor counters (``counters()``)."""
    out = {"requests": 0, "generations": 0, "errors": 0, "total_tokens_generated": 0,
           "total_processing_time": 0.0, "ttft": []}
    for p in parts:
        for k in ("requests", "generations", "errors", "total_tokens_generated",
                  "total_processing_time"):
            out[k] += p.get(k, 0)
        out["ttft"].extend(p.get("ttft", []))
    return out
