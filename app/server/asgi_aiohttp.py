"""ASGI 3 server on aiohttp (HTTP + WebSocket).

uvicorn ships no WebSocket protocol implementation in this image (neither
``websockets`` nor ``wsproto`` is installed: ``uvicorn.protocols.websockets.auto
.AutoWebSocketsProtocol is None``), so ``uvicorn.run`` would serve the HTTP routes
but reject ``/ws/llm`` upgrades.  This module hosts any ASGI app (the FastAPI
app of the WS server) on aiohttp's server, which implements RFC 6455 itself:

* ``http`` scope: request body delivered in one ``http.request`` event,
  streamed responses (SSE) written chunk by chunk;
* ``websocket`` scope: ``websocket.connect`` -> ``accept`` prepares the aiohttp
  ``WebSocketResponse``; a reader task turns frames into ``websocket.receive``
  events; ``websocket.send`` / ``close`` map to ``send_str`` / ``close``;
* ``lifespan`` startup/shutdown events are forwarded when the app handles them.
"""
from __future__ import annotations

import asyncio
import logging
from typing import Any, Awaitable, Callable, Dict, Optional

from aiohttp import WSMsgType, web

logger = logging.getLogger(__name__)

ASGIApp = Callable[[Dict[str, Any], Callable[[], Awaitable[Dict]], Callable[[Dict], Awaitable[None]]],
                   Awaitable[None]]


def _headers(request: web.Request):
    return [(k.lower(), v) for k, v in request.raw_headers]


def _base_scope(request: web.Request, kind: str) -> Dict[str, Any]:
    peer = request.transport.get_extra_info("peername") if request.transport else None
    sock = request.transport.get_extra_info("sockname") if request.transport else None
    return {
        "type": kind,
        "asgi": {"version": "3.0", "spec_version": "2.3"},
        "http_version": f"{request.version.major}.{request.version.minor}",
        "scheme": ("wss" if request.secure else "ws") if kind == "websocket" else request.scheme,
        "path": request.path,
        "raw_path": request.raw_path.split("?", 1)[0].encode(),
        "query_string": request.query_string.encode(),
        "root_path": "",
        "headers": _headers(request),
        "client": tuple(peer[:2]) if peer else None,
        "server": tuple(sock[:2]) if sock else None,
    }


class AiohttpASGIServer:
    def __init__(self, app: ASGIApp, host: str = "0.0.0.0", port: int = 8000,
                 max_msg_size: int = 16 << 20, reuse_port: bool = False):
        self.app = app
        self.host = host
        self.port = port
        self.reuse_port = reuse_port   # several worker processes on one port (app/server/workers.py)
        self.max_msg_size = max_msg_size
        self._runner: Optional[web.AppRunner] = None
        self._lifespan_q: Optional[asyncio.Queue] = None
        self._lifespan_task: Optional[asyncio.Task] = None

    # ------------------------------------------------------------------ http
    async def _http(self, request: web.Request) -> web.StreamResponse:
        body = await request.read()
        scope = _base_scope(request, "http")
        scope["method"] = request.method
        delivered = False
        disconnected = asyncio.Event()
        resp: Dict[str, Any] = {"obj": None, "status": 500, "headers": []}

        async def receive():
            nonlocal delivered
            if not delivered:
                delivered = True
                return {"type": "http.request", "body": body, "more_body": False}
            await disconnected.wait()
            return {"type": "http.disconnect"}

        async def send(msg):
            t = msg["type"]
            if t == "http.response.start":
                resp["status"] = msg["status"]
                resp["headers"] = msg.get("headers", [])
            elif t == "http.response.body":
                if resp["obj"] is None:
                    r = web.StreamResponse(status=resp["status"])
                    for k, v in resp["headers"]:
                        k = k.decode("latin-1") if isinstance(k, bytes) else k
                        v = v.decode("latin-1") if isinstance(v, bytes) else v
                        if k.lower() in ("content-length", "transfer-encoding"):
                            if k.lower() == "content-length" and not msg.get("more_body", False):
                                r.content_length = int(v)
                            continue
                        r.headers.add(k, v)
                    await r.prepare(request)
                    resp["obj"] = r
                chunk = msg.get("body", b"")
                if chunk:
                    await resp["obj"].write(chunk)
                if not msg.get("more_body", False):
                    await resp["obj"].write_eof()

        try:
            await self.app(scope, receive, send)
        finally:
            disconnected.set()
        if resp["obj"] is None:
            r = web.Response(status=resp["status"])
            return r
        return resp["obj"]

    # ------------------------------------------------------------------ websocket
    async def _websocket(self, request: web.Request) -> web.StreamResponse:
        scope = _base_scope(request, "websocket")
        proto = request.headers.get("Sec-WebSocket-Protocol", "")
        scope["subprotocols"] = [p.strip() for p in proto.split(",") if p.strip()]
        inbox: asyncio.Queue = asyncio.Queue()
        inbox.put_nowait({"type": "websocket.connect"})
        state: Dict[str, Any] = {"ws": None, "reader": None, "closed": False}
        # the app may send text frames straight on the aiohttp socket once accepted
        # (state["ws"]): the token stream skips the per-frame ASGI dict / starlette
        # layers (app/core/websocket_server_vllm.py, send)
        scope["extensions"] = {"fasttalk.aiohttp_ws": state}

        async def reader(ws: web.WebSocketResponse):
            code = 1000
            try:
                async for m in ws:
                    if m.type == WSMsgType.TEXT:
                        inbox.put_nowait({"type": "websocket.receive", "text": m.data})
                    elif m.type == WSMsgType.BINARY:
                        inbox.put_nowait({"type": "websocket.receive", "bytes": m.data})
                    elif m.type == WSMsgType.ERROR:
                        code = 1011
                        break
            finally:
                state["closed"] = True
                inbox.put_nowait({"type": "websocket.disconnect", "code": ws.close_code or code})

        async def receive():
            return await inbox.get()

        async def send(msg):
            t = msg["type"]
            if t == "websocket.accept":
                ws = web.WebSocketResponse(protocols=[msg["subprotocol"]] if msg.get("subprotocol") else (),
                                           max_msg_size=self.max_msg_size, autoping=True)
                await ws.prepare(request)
                state["ws"] = ws
                state["reader"] = asyncio.create_task(reader(ws))
            elif t == "websocket.send":
                ws = state["ws"]
                if ws is None or ws.closed:
                    raise ConnectionResetError("websocket closed")
                if msg.get("text") is not None:
                    await ws.send_str(msg["text"])
                else:
                    await ws.send_bytes(msg.get("bytes") or b"")
            elif t == "websocket.close":
                ws = state["ws"]
                if ws is None:
                    state["rejected"] = True
                elif not ws.closed:
                    await ws.close(code=msg.get("code", 1000))

        try:
            await self.app(scope, receive, send)
        except ConnectionResetError:
            pass
        finally:
            ws = state["ws"]
            if ws is not None and not ws.closed:
                await ws.close()
            if state["reader"] is not None:
                state["reader"].cancel()
                try:
                    await state["reader"]
                except (asyncio.CancelledError, Exception):
                    pass
        if state["ws"] is None:
            return web.Response(status=403, text="WebSocket connection rejected")
        return state["ws"]

    async def _dispatch(self, request: web.Request) -> web.StreamResponse:
        upgrade = request.headers.get("Upgrade", "").lower() == "websocket"
        if upgrade:
            return await self._websocket(request)
        return await self._http(request)

    # ------------------------------------------------------------------ lifespan
    async def _lifespan_startup(self):
        self._lifespan_q = asyncio.Queue()
        done = asyncio.get_running_loop().create_future()

        async def receive():
            return await self._lifespan_q.get()

        async def send(msg):
            if msg["type"] in ("lifespan.startup.complete", "lifespan.startup.failed") and not done.done():
                done.set_result(msg["type"])

        async def run():
            try:
                await self.app({"type": "lifespan", "asgi": {"version": "3.0"}}, receive, send)
            except Exception:
                if not done.done():
                    done.set_result("unsupported")

        self._lifespan_task = asyncio.create_task(run())
        await self._lifespan_q.put({"type": "lifespan.startup"})
        try:
            res = await asyncio.wait_for(done, timeout=30)
        except asyncio.TimeoutError:
            res = "timeout"
        if res == "lifespan.startup.failed":
            raise RuntimeError("ASGI lifespan startup failed")

    async def _lifespan_shutdown(self):
        if self._lifespan_q is not None:
            await self._lifespan_q.put({"type": "lifespan.shutdown"})
        if self._lifespan_task is not None:
            try:
                await asyncio.wait_for(self._lifespan_task, timeout=5)
            except (asyncio.TimeoutError, Exception):
                self._lifespan_task.cancel()

    # ------------------------------------------------------------------ run
    async def start(self, listen: bool = True):
        """``listen=False``: set the server up without a listening socket; connections
        accepted elsewhere (the DP front door, app/server/front_door.py) are adopted
        with ``loop.connect_accepted_socket(self.protocol_factory(), sock=...)``."""
        await self._lifespan_startup()
        web_app = web.Application(client_max_size=self.max_msg_size)
        web_app.router.add_route("*", "/{tail:.*}", self._dispatch)
        self._runner = web.AppRunner(web_app, access_log=None, handle_signals=False)
        await self._runner.setup()
        if not listen:
            logger.info("serving adopted connections (no listening socket)")
            return
        site = web.TCPSite(self._runner, self.host, self.port, reuse_address=True,
                           reuse_port=self.reuse_port or None)
        await site.start()
        if self.port == 0:
            for s in self._runner.sites:
                srv = getattr(s, "_server", None)
                if srv is not None and srv.sockets:
                    self.port = srv.sockets[0].getsockname()[1]
        logger.info("serving on %s:%s", self.host, self.port)

    def protocol_factory(self):
        """aiohttp's low-level server (a protocol factory) once ``start`` ran."""
        assert self._runner is not None and self._runner.server is not None
        return self._runner.server

    async def stop(self):
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None
        await self._lifespan_shutdown()

    async def serve_forever(self):
        await self.start()
        try:
            while True:
                await asyncio.sleep(3600)
        finally:
            await self.stop()


def run(app: ASGIApp, host: str = "0.0.0.0", port: int = 8000):
    """Blocking entry point (the uvicorn.run equivalent)."""
    srv = AiohttpASGIServer(app, host, port)
    try:
        asyncio.run(srv.serve_forever())
    except KeyboardInterrupt:
        pass
