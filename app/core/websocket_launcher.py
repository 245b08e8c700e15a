"""Server lifecycle (API of the reference ``app/core/websocket_launcher.py``:
``WebSocketLauncher(config).start()/stop()``).

Picks the v2 server for ``native`` / ``vllm`` / ``openai`` and the legacy v1
server for ``ollama``; verifies the backend before serving (exit 1 on failure,
like the reference); serves the FastAPI app with the aiohttp ASGI transport
(uvicorn has no WebSocket implementation in this image).  For the native
provider the engine is built (and its decode graphs warmed) before the socket
opens, so the first session does not pay for model init.
"""
from __future__ import annotations

import asyncio
import signal
import sys
from typing import Optional

from app.utils.config import Config
from app.utils.logger import get_logger

logger = get_logger(__name__)


class WebSocketLauncher:
    def __init__(self, config: Optional[Config] = None, monitor=None):
        self.config = config or Config()
        self.monitor = monitor
        self.server = None
        self.should_stop = False
        self._asgi = None
        try:
            signal.signal(signal.SIGINT, self._signal_handler)
            signal.signal(signal.SIGTERM, self._signal_handler)
        except ValueError:  # not on the main thread (tests)
            pass

    def _signal_handler(self, signum, frame):
        logger.info(f"Received signal {signum}, shutting down")
        self.should_stop = True
        sys.exit(0)

    def _create_server(self):
        if self.config.llm_provider == "ollama":
            from app.core.websocket_server import WebSocketLLMServer
        else:
            from app.core.websocket_server_vllm import WebSocketLLMServer
        return WebSocketLLMServer(self.config, monitor=self.monitor)

    def _verify_connection(self) -> bool:
        ok = self.server._check_backend_connection()
        if not ok:
            logger.error(f"Backend for provider '{self.config.llm_provider}' is not reachable")
        return ok

    def _dp_workers(self) -> int:
        c = self.config
        if c.llm_provider == "native" and int(getattr(c, "engine_dp_size", 1) or 1) > 1 and \
                getattr(c, "engine_dp_mode", "workers") == "workers":
            return int(c.engine_dp_size)
        return 0

    def start(self):
        n = self._dp_workers()
        if n:
            # N service processes on one port, one engine (GPU / TP group) each
            from app.server.workers import WorkerPool

            logger.info(f"Starting {n} DP service workers on {self.config.host}:{self.config.port}")
            import os

            self._pool = WorkerPool(n, self.config.host, self.config.port,
                                    tp=int(getattr(self.config, "engine_tp_size", 1) or 1),
                                    max_restarts=int(os.environ.get("ENGINE_MAX_RESTARTS", "3")),
                                    max_connections=self.config.max_connections)
            if self.monitor is not None and hasattr(self.monitor, "attach_node"):
                self.monitor.attach_node(self._pool.board)   # :9092 reports every worker
            self._pool.start()
            try:
                if not self._pool.wait_ready():
                    # a worker failed its backend check (or died) before serving: exit 1
                    # like the single-process launcher (reference websocket_launcher.py:105)
                    sys.exit(1)
                self._pool.run()
            except KeyboardInterrupt:
                pass
            finally:
                self._pool.stop()
                self._pool.close()
            return
        logger.info(f"Starting LLM WebSocket server (provider: {self.config.llm_provider})")
        self.server = self._create_server()
        if self.monitor is not None and hasattr(self.monitor, "attach_server"):
            self.monitor.attach_server(self.server)
        if not self._verify_connection():
            sys.exit(1)
        logger.info(f"Serving on {self.config.host}:{self.config.port} "
                    f"(model {self.config.current_model()}, max connections {self.config.max_connections})")
        from app.server.asgi_aiohttp import AiohttpASGIServer

        self._asgi = AiohttpASGIServer(self.server.app, self.config.host, self.config.port)
        try:
            asyncio.run(self._asgi.serve_forever())
        except (KeyboardInterrupt, SystemExit):
            pass

    def stop(self):
        logger.info("Stopping LLM WebSocket server")
        pool = getattr(self, "_pool", None)
        if pool is not None:
            pool.stop()
        if self.server is not None and getattr(self.server, "ollama_handler", None) is not None:
            self.server.ollama_handler.close()
        if self.server is not None and getattr(self.server, "native_handler", None) is not None:
            eng = self.server.native_handler.engine
            if hasattr(eng, "shutdown"):
                eng.shutdown()
