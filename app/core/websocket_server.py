"""Legacy v1 WebSocket server (reference ``app/core/websocket_server.py``, the
Ollama-era protocol).  Same routes minus ``/models``; v1 frame shapes:
``session_started`` = ``{session_id}``, ``session_configured`` without
``provider``, ``response_complete.stats`` with tokens_generated /
processing_time_ms / tokens_per_second only, ``/health`` reports
``ollama_connection``, no ``update_config``.  Selected by the launcher for
``LLM_PROVIDER=ollama`` (reference ``websocket_launcher.py:54-61``).
"""
from __future__ import annotations

from typing import Any, Dict

from fastapi.responses import JSONResponse

from app.core.websocket_server_vllm import WebSocketLLMServer as _V2


class WebSocketLLMServer(_V2):
    VERSION = "1.0.0"

    def __init__(self, config, monitor=None, engine=None):
        super().__init__(config, monitor=monitor, engine=engine)
        self.app.version = self.VERSION
        self._patch_routes()

    def _patch_routes(self):
        keep = []
        for r in self.app.router.routes:
            path = getattr(r, "path", "")
            if path in ("/", "/health", "/models"):
                continue
            keep.append(r)
        self.app.router.routes[:] = keep

        @self.app.get("/")
        async def root():
            return {"service": "FastTalk LLM Service", "status": "ready",
                    "model": self._current_model(), "version": self.VERSION}

        @self.app.get("/health")
        async def health():
            try:
                import asyncio

                ok = await asyncio.to_thread(self._check_backend_connection)
                body = {"status": "healthy" if ok else "degraded", "model": self._current_model(),
                        "ollama_connection": ok,
                        "active_connections": self.connection_manager.get_active_count(),
                        "active_sessions": self.conversation_manager.get_session_count()}
                return JSONResponse(content=body, status_code=200 if ok else 503)
            except Exception as e:
                return JSONResponse(content={"status": "unhealthy", "error": str(e)}, status_code=503)

    def _shape_frame(self, obj: Dict[str, Any]) -> Dict[str, Any]:
        """v1 frame shapes (reference ``websocket_server.py:160-163``, ``:232-240``), applied
        in the server's ``send`` path so they hold on every transport -- including the
        aiohttp socket the v2 hot path writes to directly."""
        t = obj.get("type")
        if t == "session_started":
            return {"type": t, "session_id": obj["session_id"]}
        if t == "session_configured":
            return {"type": t, "config": obj.get("config", {})}
        if t == "response_complete":
            s = obj.get("stats", {})
            return {"type": t, "stats": {k: s[k] for k in ("tokens_generated", "processing_time_ms",
                                                           "tokens_per_second") if k in s}}
        return obj

    async def _handle_message(self, session_id: str, message: Dict[str, Any], send):
        if message.get("type") == "update_config":
            await send({"type": "error", "error": {"code": "unknown_message_type",
                                                   "message": "Unknown message type: update_config"}})
            return
        await super()._handle_message(session_id, message, send)
