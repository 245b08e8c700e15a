"""Live WebSocket connection registry (API of the reference
``app/utils/connection_manager.py``: ``ConnectionState``, ``ConnectionInfo``,
``ConnectionManager`` with the same counters and ``get_statistics`` keys).

Appendix D Q2: ``ConnectionInfo.config`` now really holds the per-session
generation config (set by ``start_session`` / ``update_config``) and the server
honours it.
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass, field
from enum import Enum
from threading import Lock
from typing import Any, Dict, List, Optional

logger = logging.getLogger(__name__)


class ConnectionState(Enum):
    CONNECTING = "connecting"
    ACTIVE = "active"
    PROCESSING = "processing"
    DISCONNECTING = "disconnecting"
    CLOSED = "closed"


@dataclass
class ConnectionInfo:
    session_id: str
    websocket: Any
    state: ConnectionState = ConnectionState.CONNECTING
    start_time: float = field(default_factory=time.time)
    last_activity: float = field(default_factory=time.time)
    messages_received: int = 0
    messages_sent: int = 0
    tokens_generated: int = 0
    generations_completed: int = 0
    errors_count: int = 0
    config: Dict[str, Any] = field(default_factory=dict)
    conversation_history: list = field(default_factory=list)

    def update_activity(self):
        self.last_activity = time.time()

    def get_duration(self) -> float:
        return time.time() - self.start_time

    def get_idle_time(self) -> float:
        return time.time() - self.last_activity

    def to_dict(self) -> Dict[str, Any]:
        return {
            "session_id": self.session_id,
            "state": self.state.value,
            "duration_seconds": self.get_duration(),
            "idle_seconds": self.get_idle_time(),
            "messages_received": self.messages_received,
            "messages_sent": self.messages_sent,
            "tokens_generated": self.tokens_generated,
            "generations_completed": self.generations_completed,
            "errors_count": self.errors_count,
            "config": dict(self.config),
        }


_TOTALS = ("messages_received", "messages_sent", "tokens_generated", "generations_completed")


class ConnectionManager:
    """Thread-safe registry enforcing ``max_connections``; per-connection counters
    are folded into the global totals when a connection is removed."""

    def __init__(self, max_connections: int = 50, admission: Any = None):
        self.max_connections = max_connections
        # node-wide gate of the DP service workers (app/server/node_state.py): an object
        # with try_admit() / release(); None = this process is the whole service
        self.admission = admission
        self.active_connections: Dict[str, ConnectionInfo] = {}
        self._lock = Lock()
        self.total_connections = 0
        self.total_disconnections = 0
        self.total_messages_received = 0
        self.total_messages_sent = 0
        self.total_tokens_generated = 0
        self.total_generations_completed = 0

    # ------------------------------------------------------------------ lifecycle
    def add_connection(self, session_id: str, websocket: Any,
                       config: Optional[Dict[str, Any]] = None) -> Optional[ConnectionInfo]:
        with self._lock:
            if len(self.active_connections) >= self.max_connections:
                logger.warning("Max connections (%d) reached; rejecting %s", self.max_connections,
                               session_id)
                return None
            if session_id in self.active_connections:
                logger.warning("Session %s already exists; replacing it", session_id)
                del self.active_connections[session_id]
                if self.admission is not None:
                    self.admission.release()
            if self.admission is not None and not self.admission.try_admit():
                logger.warning("Max connections (%d) reached on the node; rejecting %s",
                               self.max_connections, session_id)
                return None
            info = ConnectionInfo(session_id=session_id, websocket=websocket,
                                  state=ConnectionState.ACTIVE, config=dict(config or {}))
            self.active_connections[session_id] = info
            self.total_connections += 1
            return info

    def remove_connection(self, session_id: str) -> bool:
        with self._lock:
            info = self.active_connections.pop(session_id, None)
            if info is None:
                return False
            if self.admission is not None:
                self.admission.release()
            self.total_disconnections += 1
            for name in _TOTALS:
                setattr(self, "total_" + name, getattr(self, "total_" + name) + getattr(info, name))
            return True

    def get_connection(self, session_id: str) -> Optional[ConnectionInfo]:
        with self._lock:
            return self.active_connections.get(session_id)

    def update_connection_state(self, session_id: str, state: ConnectionState) -> bool:
        with self._lock:
            info = self.active_connections.get(session_id)
            if info is None:
                return False
            info.state = state
            info.update_activity()
            return True

    def update_config(self, session_id: str, cfg: Dict[str, Any]) -> bool:
        """Merge generation settings into the session config (Appendix D Q2/Q4)."""
        with self._lock:
            info = self.active_connections.get(session_id)
            if info is None:
                return False
            info.config.update({k: v for k, v in (cfg or {}).items()})
            return True

    # ------------------------------------------------------------------ counters
    def _bump(self, session_id: str, attr: str, n: int = 1):
        with self._lock:
            info = self.active_connections.get(session_id)
            if info is not None:
                setattr(info, attr, getattr(info, attr) + n)
                info.last_activity = time.time()

    def record_message_received(self, session_id: str):
        self._bump(session_id, "messages_received")

    def record_message_sent(self, session_id: str, count: int = 1):
        self._bump(session_id, "messages_sent", count)

    def record_tokens_generated(self, session_id: str, count: int):
        self._bump(session_id, "tokens_generated", count)

    def record_generation_complete(self, session_id: str):
        self._bump(session_id, "generations_completed")

    def record_error(self, session_id: str):
        self._bump(session_id, "errors_count")

    # ------------------------------------------------------------------ queries
    def get_active_count(self) -> int:
        with self._lock:
            return len(self.active_connections)

    def get_session_list(self) -> List[str]:
        with self._lock:
            return list(self.active_connections)

    def cleanup_idle_connections(self, idle_timeout: float = 3600.0) -> int:
        with self._lock:
            stale = [sid for sid, c in self.active_connections.items()
                     if c.get_idle_time() > idle_timeout]
            for sid in stale:
                del self.active_connections[sid]
                if self.admission is not None:
                    self.admission.release()
        if stale:
            logger.info("Cleaned up %d idle connections", len(stale))
        return len(stale)

    def _summary_locked(self) -> Dict[str, Any]:
        n = len(self.active_connections)
        avg = (sum(c.get_duration() for c in self.active_connections.values()) / n) if n else 0.0
        return {
            "active_connections": n,
            "max_connections": self.max_connections,
            "utilization_percent": (n / self.max_connections * 100) if self.max_connections else 0.0,
            "total_connections": self.total_connections,
            "total_disconnections": self.total_disconnections,
            "total_messages_received": self.total_messages_received,
            "total_messages_sent": self.total_messages_sent,
            "total_tokens_generated": self.total_tokens_generated,
            "total_generations_completed": self.total_generations_completed,
            "average_session_duration_seconds": avg,
        }

    def get_statistics(self) -> Dict[str, Any]:
        with self._lock:
            return self._summary_locked()

    def get_detailed_stats(self) -> Dict[str, Any]:
        with self._lock:
            return {
                "summary": self._summary_locked(),
                "active_sessions": {sid: c.to_dict() for sid, c in self.active_connections.items()},
            }

    def reset_statistics(self):
        with self._lock:
            self.total_connections = len(self.active_connections)
            self.total_disconnections = 0
            for name in _TOTALS:
                setattr(self, "total_" + name, 0)
