"""Primary FastAPI WebSocket server (v2): ``/ws/llm`` token streaming plus
``/``, ``/health``, ``/stats``, ``/models`` -- the wire protocol of the reference
``app/core/websocket_server_vllm.py`` with the
in-process MI355X engine as the default backend.

Provider dispatch:
  native (default)  -> NativeHandler (in-process AsyncEngine), optionally wrapped by
                       the native VoiceAgent (tool calling) when ENABLE_PYDANTIC_AI
  vllm / openai     -> remote OpenAI-compatible server (VLLMHandler), optionally
                       wrapped by VoiceAgent
  ollama            -> OllamaHandler (sync generator run in a worker thread)

Behavioural fixes vs the reference (Appendix D): per-session generation config
from ``start_session`` / ``update_config`` is honoured (Q2); a reader task keeps
receiving while a response streams, so ``cancel`` interrupts it (Q3);
``temperature=0`` means greedy (Q5); ``tokens_generated`` counts engine tokens
and ``response_complete`` adds ``ttft_ms`` (Q6); ``/health`` is in-process and
non-blocking (Q8); the monitoring counters are fed (Q9); ``LLMServiceError``
frames carry ``code`` and are counted (Q11); a ``user_message`` before
``start_session`` opens a session with the default system prompt (Q1).
"""
from __future__ import annotations

import asyncio
import json
import time
import uuid
from typing import Any, Dict, Optional

from fastapi import FastAPI, WebSocket, WebSocketDisconnect
from fastapi.middleware.cors import CORSMiddleware
from fastapi.responses import JSONResponse

from app.core.conversation_manager import ConversationManager
from app.utils.config import Config
from app.utils.connection_manager import ConnectionManager, ConnectionState
from app.utils.error_handler import ErrorHandler, LLMServiceError
from app.utils.logger import get_logger

logger = get_logger(__name__)

GEN_KEYS = ("temperature", "max_tokens", "top_p", "top_k", "stop", "seed", "min_tokens",
            "ignore_eos")
AGENT_KEYS = ("enable_web_search", "enable_tools", "system_prompt", "vllm_model", "vllm_base_url")


class _Turn:
    """Bookkeeping of one streamed response."""

    def __init__(self):
        self.tokens = 0
        self.text = []
        self.ttft: Optional[float] = None
        self.last_emit: Optional[float] = None
        self.engine_ttft: Optional[float] = None
        self.itl_sum = 0.0   # inter-token gaps between token frames (s)
        self.itl_n = 0
        self.finish_reason: Optional[str] = None
        self.prompt_tokens = 0
        self.cached_tokens = 0
        self.frames = 0            # token frames not yet folded into the connection stats
        self.tokens_recorded = 0


class WebSocketLLMServer:
    def __init__(self, config: Config, monitor=None, engine=None):
        self.config = config
        self.monitor = monitor
        self.app = FastAPI(title="FastTalk LLM Service",
                           description="WebSocket LLM streaming on an in-process MI355X engine",
                           version="2.0.0")
        self.app.add_middleware(CORSMiddleware, allow_origins=["*"], allow_credentials=True,
                                allow_methods=["*"], allow_headers=["*"])
        self.connection_manager = ConnectionManager(max_connections=config.max_connections)
        self.conversation_manager = ConversationManager(max_history_length=config.max_history_length)
        self.error_handler = ErrorHandler()
        self.voice_agent = None
        self.vllm_handler = None
        self.native_handler = None
        self.ollama_handler = None
        self.use_pydantic_ai = False
        self._engine = engine
        # DP service workers (app/server/workers.py): the node board makes /health and
        # /stats describe the whole node; None = this process is the whole service
        self.node = None
        self.node_index: Optional[int] = None
        self._init_llm_handler()
        self._register_routes()

    # ------------------------------------------------------------------ backends
    @property
    def provider(self) -> str:
        return self.config.llm_provider

    def _init_llm_handler(self):
        p = self.provider
        if p == "native":
            from app.core.native_handler import NativeHandler

            self.native_handler = NativeHandler(self.config, engine=self._engine,
                                                default_max_tokens=self.config.default_max_tokens)
            backend = self.native_handler
        elif p in ("vllm", "openai"):
            from app.core.vllm_handler import VLLMHandler

            self.vllm_handler = VLLMHandler(base_url=self.config.vllm_base_url,
                                            model=self.config.vllm_model,
                                            api_key=self.config.vllm_api_key,
                                            timeout=self.config.vllm_timeout)
            backend = self.vllm_handler
        else:
            from app.core.ollama_handler import OllamaHandler

            self.ollama_handler = OllamaHandler(base_url=self.config.ollama_base_url,
                                                model=self.config.model_name,
                                                keep_alive=self.config.ollama_keep_alive,
                                                timeout=self.config.ollama_timeout)
            return
        if self.config.enable_pydantic_ai:
            from app.agents.voice_agent import AgentConfig, VoiceAgent

            agent_cfg = AgentConfig(
                vllm_base_url=self.config.vllm_base_url, vllm_model=self.config.current_model(),
                vllm_api_key=self.config.vllm_api_key, temperature=self.config.default_temperature,
                max_tokens=self.config.default_max_tokens, top_p=self.config.default_top_p,
                enable_web_search=self.config.enable_web_search,
                enable_tools=self.config.enable_tools, system_prompt=self.config.system_prompt,
                guided_tool_calls=self.config.agent_json_tool_calls)
            self.voice_agent = VoiceAgent(config=agent_cfg, backend=backend)
            self.use_pydantic_ai = True

    def _current_model(self) -> str:
        return self.config.current_model()

    def _check_backend_connection(self) -> bool:
        try:
            if self.native_handler is not None:
                return self.native_handler.check_connection()
            if self.vllm_handler is not None:
                return self.vllm_handler.check_connection()
            return self.ollama_handler.check_connection()
        except Exception as e:
            logger.error(f"Backend connection check failed: {e}")
            return False

    # ------------------------------------------------------------------ routes
    def _register_routes(self):
        app = self.app

        @app.get("/")
        async def root():
            agentic = self.provider != "ollama"
            return {
                "service": "FastTalk LLM Service", "status": "ready", "version": "2.0.0",
                "provider": self.provider, "model": self._current_model(),
                "pydantic_ai_enabled": self.use_pydantic_ai,
                "web_search_enabled": self.config.enable_web_search if agentic else False,
                "tools_enabled": self.config.enable_tools if agentic else False,
            }

        @app.get("/health")
        async def health():
            try:
                if self.native_handler is not None:
                    ok = self._check_backend_connection()  # in-process, non-blocking
                else:
                    ok = await asyncio.to_thread(self._check_backend_connection)
                body = {
                    "status": "healthy" if ok else "degraded", "provider": self.provider,
                    "model": self._current_model(), "backend_connection": ok,
                    "pydantic_ai_enabled": self.use_pydantic_ai,
                    "active_connections": self.connection_manager.get_active_count(),
                    "active_sessions": self.conversation_manager.get_session_count(),
                }
                if self.node is not None:
                    # one service: healthy only while every worker is up and serving
                    workers = self.node.workers()
                    node_ok = all(w["alive"] and w["ready"] and w["heartbeat_fresh"]
                                  and w["backend_ok"] for w in workers)
                    ok = ok and node_ok
                    body["status"] = "healthy" if ok else "degraded"
                    body["active_connections"] = self.node.node_active()
                    body["worker"] = self.node_index
                    body["workers"] = workers
                return JSONResponse(content=body, status_code=200 if ok else 503)
            except Exception as e:
                return JSONResponse(content={"status": "unhealthy", "error": str(e)}, status_code=503)

        @app.get("/stats")
        async def stats():
            body = {
                "connections": self.connection_manager.get_statistics(),
                "conversations": self.conversation_manager.get_statistics(),
                "errors": self.error_handler.get_error_stats(),
                "provider": self.provider,
                "pydantic_ai_enabled": self.use_pydantic_ai,
            }
            if self.node is not None:
                from app.server.node_state import merge_service_stats

                alive = {w["index"] for w in self.node.workers() if w["alive"]}
                parts = [body] + [s for s in self.node.snapshots()
                                  if s and s.get("index") != self.node_index
                                  and s.get("index") in alive]
                body.update(merge_service_stats(parts, self.node.max_connections,
                                                active=self.node.node_active()))
                body["workers"] = self.node.workers()
            eng = self.engine_metrics()
            if eng is not None:
                body["engine"] = eng
            return body

        @app.get("/models")
        async def list_models():
            try:
                if self.voice_agent is not None:
                    return self.voice_agent.get_model_info()
                if self.native_handler is not None:
                    return self.native_handler.get_model_info()
                if self.vllm_handler is not None:
                    return await asyncio.to_thread(self.vllm_handler.get_model_info)
                return await asyncio.to_thread(self.ollama_handler.get_model_info)
            except Exception as e:
                return {"error": str(e)}

        @app.websocket("/ws/llm")
        async def websocket_endpoint(websocket: WebSocket):
            await self.handle_websocket(websocket)

        if self.native_handler is not None:
            from app.core.openai_api import register_openai_routes

            register_openai_routes(app, self.native_handler)

    def engine_metrics(self) -> Optional[Dict[str, Any]]:
        if self.native_handler is None:
            return None
        eng = self.native_handler.engine
        inner = getattr(eng, "engine", None)
        if inner is not None and hasattr(inner, "metrics"):
            return inner.metrics()
        if hasattr(eng, "metrics"):
            return eng.metrics()
        return None

    # ------------------------------------------------------------------ websocket
    async def handle_websocket(self, websocket: WebSocket):
        session_id = str(uuid.uuid4())
        await websocket.accept()
        send_lock = asyncio.Lock()
        # the aiohttp transport hands out its socket (app/server/asgi_aiohttp.py): text
        # frames go out directly instead of through starlette + the ASGI bridge, the
        # per-token cost that bounds one process's stream rate (bench/dp_ceiling.py)
        raw = (websocket.scope.get("extensions") or {}).get("fasttalk.aiohttp_ws")

        shape = self._shape_frame

        async def send(obj: Any):
            # frames are shaped here, on the one path every transport shares (the v1
            # server trims v2 frames to its shapes; token frames arrive pre-serialised)
            txt = obj if isinstance(obj, str) else json.dumps(shape(obj))
            ws = raw.get("ws") if raw is not None else None
            if ws is not None:
                # aiohttp writes each frame whole, synchronously, before any drain await,
                # so concurrent senders cannot split a frame: no lock on the per-token path
                if ws.closed:
                    raise WebSocketDisconnect(1006)
                await ws.send_str(txt)
                return
            async with send_lock:
                await websocket.send_text(txt)

        if self.connection_manager.add_connection(session_id, websocket) is None:
            await send({"type": "error", "error": {"code": "max_connections",
                                                   "message": "Maximum connections reached",
                                                   "severity": "high"}})
            await websocket.close()
            return
        work: "asyncio.Queue" = asyncio.Queue()
        state = {"task": None}

        async def worker():
            while True:
                msg = await work.get()
                if msg is None:
                    return
                try:
                    await self._handle_user_message(session_id, msg, send)
                except Exception as e:  # pragma: no cover - defensive
                    logger.error(f"[{session_id}] worker error: {e}")

        state["task"] = asyncio.create_task(worker())
        try:
            await send({"type": "session_started", "session_id": session_id,
                        "provider": self.provider, "model": self._current_model(),
                        "pydantic_ai_enabled": self.use_pydantic_ai})
            while True:
                data = await websocket.receive_text()
                self.connection_manager.record_message_received(session_id)
                try:
                    message = json.loads(data)
                    if not isinstance(message, dict):
                        raise json.JSONDecodeError("not an object", data, 0)
                except json.JSONDecodeError:
                    await send({"type": "error", "error": {"code": "invalid_json",
                                                           "message": "Invalid JSON format"}})
                    continue
                try:
                    mtype = message.get("type")
                    if mtype == "user_message":
                        if self.monitor is not None:
                            self.monitor.record_request()
                        await work.put(message)
                    else:
                        await self._handle_message(session_id, message, send)
                except Exception as e:
                    self.connection_manager.record_error(session_id)
                    info = self.error_handler.handle_error(e, {"session_id": session_id})
                    if self.monitor is not None:
                        self.monitor.record_error()
                    await send({"type": "error", "error": {
                        "code": info.category.value, "message": info.message,
                        "severity": info.severity.value, "recoverable": info.recoverable}})
        except WebSocketDisconnect:
            pass
        except Exception as e:
            logger.error(f"[{session_id}] Unexpected error: {e}")
        finally:
            self._cancel_active(session_id)
            await work.put(None)
            t = state["task"]
            if t is not None:
                t.cancel()
                try:
                    await t
                except (asyncio.CancelledError, Exception):
                    pass
            self.connection_manager.remove_connection(session_id)
            self.conversation_manager.end_session(session_id)
            if self.native_handler is not None:
                self.native_handler.forget_session(session_id)

    def _shape_frame(self, obj: Dict[str, Any]) -> Dict[str, Any]:
        """Protocol-version hook on every outgoing control frame (v2: unchanged)."""
        return obj

    async def _handle_message(self, session_id: str, message: Dict[str, Any], send):
        t = message.get("type")
        if t == "start_session":
            await self._handle_start_session(session_id, message, send)
        elif t == "cancel":
            await self._handle_cancel(session_id, send)
        elif t == "end_session":
            await self._handle_end_session(session_id, send)
        elif t == "update_config":
            await self._handle_update_config(session_id, message, send)
        else:
            await send({"type": "error", "error": {"code": "unknown_message_type",
                                                   "message": f"Unknown message type: {t}"}})

    async def _handle_start_session(self, session_id: str, message: Dict[str, Any], send):
        cfg = message.get("config") or {}
        if not isinstance(cfg, dict):
            cfg = {}
        self.conversation_manager.create_session(session_id=session_id,
                                                 system_prompt=cfg.get("system_prompt"))
        self.connection_manager.update_config(session_id, {k: cfg[k] for k in GEN_KEYS if k in cfg})
        await send({"type": "session_configured", "config": cfg, "provider": self.provider})
        self.connection_manager.record_message_sent(session_id)

    def _gen_settings(self, session_id: str) -> Dict[str, Any]:
        info = self.connection_manager.get_connection(session_id)
        sc = dict(info.config) if info else {}
        c = self.config
        out = {
            "temperature": sc.get("temperature", c.default_temperature),
            "max_tokens": sc.get("max_tokens", c.default_max_tokens),
            "top_p": sc.get("top_p", c.default_top_p),
            # vLLM-path parity: top_k only when the session asks for it (Ollama sends DEFAULT_TOP_K)
            "top_k": sc.get("top_k", c.default_top_k if self.provider == "ollama" else None),
        }
        for k in ("stop", "seed", "min_tokens", "ignore_eos"):
            if k in sc:
                out[k] = sc[k]
        return out

    async def _handle_user_message(self, session_id: str, message: Dict[str, Any], send):
        text = message.get("text", "")
        if not text or not isinstance(text, str):
            await send({"type": "error", "error": {"code": "empty_message",
                                                   "message": "Empty user message"}})
            return
        if not self.conversation_manager.has_session(session_id):
            self.conversation_manager.create_session(session_id, system_prompt=self.config.system_prompt)
        self.conversation_manager.add_user_message(session_id, text)
        self.connection_manager.update_connection_state(session_id, ConnectionState.PROCESSING)
        t0 = time.time()
        turn = _Turn()
        try:
            async with self.error_handler.generation_circuit_breaker.guard():
                if self.use_pydantic_ai:
                    await self._generate_with_agent(session_id, text, send, turn)
                elif self.native_handler is not None:
                    await self._generate_with_native(session_id, send, turn)
                elif self.vllm_handler is not None:
                    await self._generate_with_vllm(session_id, send, turn)
                else:
                    await self._generate_with_ollama(session_id, send, turn)
            dur = time.time() - t0
            full = "".join(turn.text)
            self.conversation_manager.add_assistant_message(session_id, full, tokens_generated=turn.tokens)
            self.connection_manager.record_generation_complete(session_id)
            if self.monitor is not None:
                self.monitor.record_generation(turn.tokens, dur, ttft=turn.ttft)
            stats = {
                "tokens_generated": turn.tokens,
                "processing_time_ms": dur * 1000.0,
                "tokens_per_second": turn.tokens / dur if dur > 0 else 0.0,
                "provider": self.provider,
                "pydantic_ai_used": self.use_pydantic_ai,
            }
            if turn.ttft is not None:
                stats["ttft_ms"] = turn.ttft * 1000.0
            if turn.itl_n:
                stats["itl_ms"] = 1000.0 * turn.itl_sum / turn.itl_n
            if turn.engine_ttft is not None:
                stats["engine_ttft_ms"] = 1000.0 * turn.engine_ttft
            if turn.finish_reason is not None:
                stats["finish_reason"] = turn.finish_reason
            if turn.prompt_tokens:
                stats["prompt_tokens"] = turn.prompt_tokens
                stats["cached_prompt_tokens"] = turn.cached_tokens
            self._flush_turn_stats(session_id, turn)
            await send({"type": "response_complete", "stats": stats})
            self.connection_manager.record_message_sent(session_id)
        except LLMServiceError as e:
            self.error_handler.handle_error(e, {"session_id": session_id})
            self.connection_manager.record_error(session_id)
            if self.monitor is not None:
                self.monitor.record_error()
            await send({"type": "error", "error": e.to_dict()})
        except Exception as e:
            info = self.error_handler.handle_error(e, {"session_id": session_id})
            self.connection_manager.record_error(session_id)
            if self.monitor is not None:
                self.monitor.record_error()
            await send({"type": "error", "error": {"code": info.category.value, "message": info.message,
                                                   "severity": info.severity.value}})
        finally:
            self._flush_turn_stats(session_id, turn)
            self.connection_manager.update_connection_state(session_id, ConnectionState.ACTIVE)

    async def _emit(self, session_id: str, send, turn: _Turn, text: str, ntok: int, t_start: float):
        now = time.time()
        if turn.ttft is None:
            turn.ttft = now - t_start
        elif turn.last_emit is not None:
            turn.itl_sum += now - turn.last_emit
            turn.itl_n += 1
        turn.last_emit = now
        turn.tokens += ntok
        if text:
            turn.text.append(text)
            # the frame {"type": "token", "data": ...} json.dumps would write
            await send('{"type": "token", "data": ' + json.dumps(text) + "}")
            turn.frames += 1
        # connection counters are folded in once per turn (_flush_turn_stats)

    def _flush_turn_stats(self, session_id: str, turn: _Turn):
        if turn.frames:
            self.connection_manager.record_message_sent(session_id, turn.frames)
        n = turn.tokens - turn.tokens_recorded
        if n:
            self.connection_manager.record_tokens_generated(session_id, n)
        turn.frames = 0
        turn.tokens_recorded = turn.tokens

    async def _generate_with_native(self, session_id: str, send, turn: _Turn):
        messages = self.conversation_manager.get_messages_for_generation(session_id) or []
        g = self._gen_settings(session_id)
        t0 = time.time()
        async for out in self.native_handler.stream_events(
                messages, temperature=g["temperature"], max_tokens=g["max_tokens"], top_p=g["top_p"],
                top_k=g["top_k"], stop=g.get("stop"), request_id=session_id, session_id=session_id,
                seed=g.get("seed"), ignore_eos=bool(g.get("ignore_eos", False)),
                min_tokens=int(g.get("min_tokens", 0) or 0)):
            if out.token_ids or out.text:
                await self._emit(session_id, send, turn, out.text, len(out.token_ids), t0)
            if out.ttft_s is not None and turn.engine_ttft is None:
                turn.engine_ttft = out.ttft_s
            if out.num_prompt_tokens:
                turn.prompt_tokens = out.num_prompt_tokens
                turn.cached_tokens = out.num_cached_tokens
            if out.finished:
                turn.finish_reason = out.finish_reason

    async def _generate_with_agent(self, session_id: str, user_text: str, send, turn: _Turn):
        from datetime import datetime

        from app.agents.voice_agent import ConversationContext

        history = self.conversation_manager.get_messages_for_generation(session_id) or []
        ctx = ConversationContext(user_id=session_id, session_id=session_id,
                                  conversation_history=[{"role": m["role"], "content": m["content"]}
                                                        for m in history[:-1]],
                                  created_at=datetime.now())
        g = self._gen_settings(session_id)
        t0 = time.time()
        async for ev in self.voice_agent.generate_events(
                user_message=user_text, context=ctx, temperature=g["temperature"],
                max_tokens=g["max_tokens"], top_p=g["top_p"], top_k=g["top_k"], stop=g.get("stop"),
                seed=g.get("seed"), ignore_eos=bool(g.get("ignore_eos", False)),
                min_tokens=int(g.get("min_tokens", 0) or 0)):
            if ev.text or ev.num_tokens:
                await self._emit(session_id, send, turn, ev.text, ev.num_tokens, t0)
            if ev.engine_ttft_s is not None and turn.engine_ttft is None:
                turn.engine_ttft = ev.engine_ttft_s
            if ev.prompt_tokens:
                turn.prompt_tokens = ev.prompt_tokens
                turn.cached_tokens = ev.cached_tokens
            if ev.finish_reason:
                turn.finish_reason = ev.finish_reason

    async def _generate_with_vllm(self, session_id: str, send, turn: _Turn):
        messages = self.conversation_manager.get_messages_for_generation(session_id) or []
        g = self._gen_settings(session_id)
        t0 = time.time()
        async for tok in self.vllm_handler.generate_stream_async(
                messages=messages, temperature=g["temperature"], max_tokens=g["max_tokens"],
                top_p=g["top_p"], stop=g.get("stop"), request_id=session_id):
            await self._emit(session_id, send, turn, tok, 1, t0)

    async def _generate_with_ollama(self, session_id: str, send, turn: _Turn):
        messages = self.conversation_manager.get_messages_for_generation(session_id) or []
        g = self._gen_settings(session_id)
        gen = self.ollama_handler.generate_stream(
            messages=messages, temperature=g["temperature"], max_tokens=g["max_tokens"],
            top_p=g["top_p"], top_k=g["top_k"], stop=g.get("stop"), request_id=session_id)
        loop = asyncio.get_running_loop()
        q: "asyncio.Queue" = asyncio.Queue()
        sentinel = object()

        def pump():
            try:
                for tok in gen:
                    loop.call_soon_threadsafe(q.put_nowait, tok)
            except BaseException as e:  # forwarded to the coroutine
                loop.call_soon_threadsafe(q.put_nowait, e)
            finally:
                loop.call_soon_threadsafe(q.put_nowait, sentinel)

        fut = loop.run_in_executor(None, pump)
        t0 = time.time()
        while True:
            item = await q.get()
            if item is sentinel:
                break
            if isinstance(item, BaseException):
                raise item
            await self._emit(session_id, send, turn, item, 1, t0)
        await fut

    def _cancel_active(self, session_id: str) -> bool:
        if self.native_handler is not None:
            ok = self.native_handler.cancel_generation(session_id)
            if self.voice_agent is not None:
                ok = self.voice_agent.cancel(session_id) or ok
            return ok
        if self.vllm_handler is not None:
            return self.vllm_handler.cancel_generation(session_id)
        if self.ollama_handler is not None:
            return self.ollama_handler.cancel_generation(session_id)
        return False

    async def _handle_cancel(self, session_id: str, send):
        ok = self._cancel_active(session_id)
        await send({"type": "cancelled", "success": ok})
        self.connection_manager.record_message_sent(session_id)

    async def _handle_end_session(self, session_id: str, send):
        info = self.connection_manager.get_connection(session_id)
        await send({"type": "session_ended", "stats": info.to_dict() if info else {}})
        self.connection_manager.record_message_sent(session_id)

    async def _handle_update_config(self, session_id: str, message: Dict[str, Any], send):
        cfg = message.get("config") or {}
        if not isinstance(cfg, dict):
            cfg = {}
        self.connection_manager.update_config(session_id, {k: cfg[k] for k in GEN_KEYS if k in cfg})
        agent_level = {k: v for k, v in cfg.items() if k in AGENT_KEYS}
        if self.voice_agent is not None and agent_level:
            self.voice_agent.update_config(**agent_level)
        await send({"type": "config_updated", "success": True, "config": cfg})
        self.connection_manager.record_message_sent(session_id)
