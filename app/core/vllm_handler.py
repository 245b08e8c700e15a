"""Remote OpenAI-compatible backend (``LLM_PROVIDER=vllm|openai``).

Same public surface as the reference ``app/core/vllm_handler.py`` (``VLLMHandler``
and ``VLLMWithToolsHandler``), but implemented directly on ``httpx`` against
``/v1/chat/completions`` with ``stream=true`` (SSE) -- the ``openai`` SDK is not
a dependency of this image.  Useful to front an external engine (vLLM-ROCm, or
another instance of this service's OpenAI facade ``/v1``).
"""
from __future__ import annotations

import json
import logging
import time
import uuid
from threading import Lock
from typing import Any, AsyncGenerator, Callable, Dict, Generator, List, Optional

import httpx

from app.utils.error_handler import ErrorCategory, ErrorSeverity, LLMServiceError

logger = logging.getLogger(__name__)


def _sse_payloads(lines):
    for line in lines:
        if not line or not line.startswith("data:"):
            continue
        data = line[5:].strip()
        if data == "[DONE]":
            return
        try:
            yield json.loads(data)
        except json.JSONDecodeError:
            logger.warning("bad SSE payload: %s", data[:80])


class VLLMHandler:
    def __init__(self, base_url: str, model: str, api_key: str = "not-needed", timeout: float = 600.0):
        self.base_url = base_url.rstrip("/")
        self.model = model
        self.api_key = api_key
        self.timeout = timeout
        self._headers = {"Authorization": f"Bearer {api_key}", "Content-Type": "application/json"}
        self._active_requests: Dict[str, Dict[str, Any]] = {}
        self._requests_lock = Lock()
        self._connection_ok = False

    # ------------------------------------------------------------------ health / info
    def _health_url(self) -> str:
        return self.base_url[:-3] + "/health" if self.base_url.endswith("/v1") else self.base_url + "/health"

    def check_connection(self) -> bool:
        try:
            with httpx.Client(timeout=5.0) as c:
                c.get(self._health_url()).raise_for_status()
            self._connection_ok = True
        except Exception as e:
            logger.error("Failed to connect to %s: %s", self.base_url, e)
            self._connection_ok = False
        return self._connection_ok

    def get_model_info(self) -> Dict[str, Any]:
        try:
            with httpx.Client(timeout=10.0, headers=self._headers) as c:
                r = c.get(self.base_url + "/models")
                r.raise_for_status()
                return {"models": [m["id"] for m in r.json().get("data", [])], "current_model": self.model}
        except Exception as e:
            raise LLMServiceError(f"Failed to get model info: {e}", category=ErrorCategory.CONNECTION,
                                  severity=ErrorSeverity.MEDIUM)

    # ------------------------------------------------------------------ request tracking
    def _params(self, messages, temperature, max_tokens, top_p, stop, tools,
                tool_choice=None, extra: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        body: Dict[str, Any] = {"model": self.model, "messages": messages, "stream": True}
        for k, v in (("temperature", temperature), ("max_tokens", max_tokens), ("top_p", top_p),
                     ("stop", stop), ("tools", tools)):
            if v is not None:
                body[k] = v
        if tools and tool_choice is not None:
            body["tool_choice"] = tool_choice
        for k, v in (extra or {}).items():   # vLLM sampling extensions: top_k, seed, ignore_eos ...
            if v is not None:
                body[k] = v
        return body

    def _register(self, req_id: str):
        with self._requests_lock:
            self._active_requests[req_id] = {"start_time": time.time(), "cancelled": False}

    def _cancelled(self, req_id: str) -> bool:
        with self._requests_lock:
            info = self._active_requests.get(req_id)
            return info is None or info["cancelled"]

    def _unregister(self, req_id: str):
        with self._requests_lock:
            self._active_requests.pop(req_id, None)

    @staticmethod
    def _delta(chunk) -> (Optional[str], Optional[str]):
        ch = (chunk.get("choices") or [{}])[0]
        return (ch.get("delta") or {}).get("content"), ch.get("finish_reason")

    # ------------------------------------------------------------------ streaming
    def generate_stream(self, messages: List[Dict[str, str]], temperature: Optional[float] = None,
                        max_tokens: Optional[int] = None, top_p: Optional[float] = None,
                        stop: Optional[List[str]] = None, tools: Optional[List[Dict]] = None,
                        request_id: Optional[str] = None) -> Generator[str, None, None]:
        req_id = request_id or f"vllm-{uuid.uuid4()}"
        self._register(req_id)
        try:
            with httpx.Client(timeout=self.timeout, headers=self._headers) as c:
                with c.stream("POST", self.base_url + "/chat/completions",
                              json=self._params(messages, temperature, max_tokens, top_p, stop, tools)) as r:
                    r.raise_for_status()
                    for chunk in _sse_payloads(r.iter_lines()):
                        if self._cancelled(req_id):
                            break
                        text, fin = self._delta(chunk)
                        if text:
                            yield text
                        if fin:
                            break
        except LLMServiceError:
            raise
        except Exception as e:
            raise LLMServiceError(f"vLLM generation error: {e}", category=ErrorCategory.PROCESSING,
                                  severity=ErrorSeverity.HIGH)
        finally:
            self._unregister(req_id)

    async def generate_stream_async(self, messages: List[Dict[str, str]], temperature: Optional[float] = None,
                                    max_tokens: Optional[int] = None, top_p: Optional[float] = None,
                                    stop: Optional[List[str]] = None, tools: Optional[List[Dict]] = None,
                                    request_id: Optional[str] = None) -> AsyncGenerator[str, None]:
        req_id = request_id or f"vllm-async-{uuid.uuid4()}"
        self._register(req_id)
        try:
            async with httpx.AsyncClient(timeout=self.timeout, headers=self._headers) as c:
                async with c.stream("POST", self.base_url + "/chat/completions",
                                    json=self._params(messages, temperature, max_tokens, top_p, stop, tools)) as r:
                    r.raise_for_status()
                    async for line in r.aiter_lines():
                        if self._cancelled(req_id):
                            break
                        for chunk in _sse_payloads([line]):
                            text, fin = self._delta(chunk)
                            if text:
                                yield text
                            if fin:
                                return
        except LLMServiceError:
            raise
        except Exception as e:
            raise LLMServiceError(f"vLLM async generation error: {e}", category=ErrorCategory.PROCESSING,
                                  severity=ErrorSeverity.HIGH)
        finally:
            self._unregister(req_id)

    async def stream_chat_async(self, messages: List[Dict[str, Any]], temperature: Optional[float] = None,
                                max_tokens: Optional[int] = None, top_p: Optional[float] = None,
                                stop: Optional[List[str]] = None, tools: Optional[List[Dict]] = None,
                                tool_choice: Any = None, request_id: Optional[str] = None,
                                extra: Optional[Dict[str, Any]] = None
                                ) -> AsyncGenerator[Dict[str, Any], None]:
        """One streamed chat completion with tools (what the reference's PydanticAI
        agent sends, ``/root/reference/app/agents/voice_agent.py:219``): yields
        ``{"type": "text", "text"}`` per content delta, then -- when the server
        answered with calls -- one ``{"type": "tool_calls", "calls": [{"id",
        "name", "arguments"}]}`` assembled from the streamed ``tool_calls`` deltas
        (keyed by ``index``; the id and name come first, argument fragments after),
        and finally ``{"type": "finish", "reason"}``."""
        req_id = request_id or f"vllm-chat-{uuid.uuid4()}"
        self._register(req_id)
        calls: Dict[int, Dict[str, Any]] = {}
        finish = None
        try:
            async with httpx.AsyncClient(timeout=self.timeout, headers=self._headers) as c:
                body = self._params(messages, temperature, max_tokens, top_p, stop, tools,
                                    tool_choice, extra)
                async with c.stream("POST", self.base_url + "/chat/completions", json=body) as r:
                    r.raise_for_status()
                    async for line in r.aiter_lines():
                        if self._cancelled(req_id):
                            finish = "abort"
                            break
                        for chunk in _sse_payloads([line]):
                            ch = (chunk.get("choices") or [{}])[0]
                            delta = ch.get("delta") or {}
                            if delta.get("content"):
                                yield {"type": "text", "text": delta["content"]}
                            for tc in delta.get("tool_calls") or []:
                                slot = calls.setdefault(int(tc.get("index", len(calls))),
                                                        {"id": None, "name": None, "arguments": ""})
                                if tc.get("id"):
                                    slot["id"] = tc["id"]
                                fn = tc.get("function") or {}
                                if fn.get("name"):
                                    slot["name"] = fn["name"]
                                if fn.get("arguments"):
                                    slot["arguments"] += fn["arguments"]
                            if ch.get("finish_reason"):
                                finish = ch["finish_reason"]
        except LLMServiceError:
            raise
        except Exception as e:
            raise LLMServiceError(f"vLLM chat error: {e}", category=ErrorCategory.PROCESSING,
                                  severity=ErrorSeverity.HIGH)
        finally:
            self._unregister(req_id)
        if calls:
            out = []
            for i in sorted(calls):
                cinfo = calls[i]
                out.append({"id": cinfo["id"] or f"call_{uuid.uuid4().hex[:12]}",
                            "name": cinfo["name"], "arguments": cinfo["arguments"]})
            yield {"type": "tool_calls", "calls": out}
        yield {"type": "finish", "reason": finish or "stop"}

    def cancel_generation(self, request_id: str) -> bool:
        with self._requests_lock:
            info = self._active_requests.get(request_id)
            if info is None:
                return False
            info["cancelled"] = True
            return True

    def get_active_requests(self) -> Dict[str, Dict[str, Any]]:
        now = time.time()
        with self._requests_lock:
            return {k: {"start_time": v["start_time"], "duration_s": now - v["start_time"],
                        "cancelled": v["cancelled"]} for k, v in self._active_requests.items()}


class VLLMWithToolsHandler(VLLMHandler):
    """Client-side tool loop: accumulate streamed ``tool_calls``, run the Python
    callables, append assistant/tool messages and stream the continuation."""

    def generate_stream_with_tools(self, messages: List[Dict[str, Any]], tools: List[Dict],
                                   tool_functions: Dict[str, Callable], temperature: Optional[float] = None,
                                   max_tokens: Optional[int] = None, request_id: Optional[str] = None,
                                   max_rounds: int = 4) -> Generator[str, None, None]:
        req_id = request_id or f"vllm-tools-{uuid.uuid4()}"
        for _ in range(max_rounds):
            # streamed tool_calls deltas are keyed by `index` (OpenAI / vLLM): the first
            # delta of a call carries its id and name, later ones argument fragments
            calls: Dict[int, Dict[str, Any]] = {}
            body = self._params(messages, temperature, max_tokens, None, None, tools)
            with httpx.Client(timeout=self.timeout, headers=self._headers) as c:
                with c.stream("POST", self.base_url + "/chat/completions", json=body) as r:
                    r.raise_for_status()
                    for chunk in _sse_payloads(r.iter_lines()):
                        delta = ((chunk.get("choices") or [{}])[0].get("delta") or {})
                        for tc in delta.get("tool_calls") or []:
                            slot = calls.setdefault(int(tc.get("index", len(calls))),
                                                    {"id": None, "name": None, "arguments": ""})
                            if tc.get("id"):
                                slot["id"] = tc["id"]
                            fn = tc.get("function") or {}
                            if fn.get("name"):
                                slot["name"] = fn["name"]
                            if fn.get("arguments"):
                                slot["arguments"] += fn["arguments"]
                        if delta.get("content"):
                            yield delta["content"]
            if not calls:
                return
            for i in sorted(calls):
                info = calls[i]
                cid = info["id"] or f"call_{uuid.uuid4().hex[:12]}"
                fn = tool_functions.get(info["name"])
                if fn is None:
                    continue
                try:
                    result = fn(**json.loads(info["arguments"] or "{}"))
                except Exception as e:  # surfaced inline like the reference
                    yield f"\n[Error executing tool: {e}]"
                    return
                messages.append({"role": "assistant", "tool_calls": [
                    {"id": cid, "type": "function",
                     "function": {"name": info["name"], "arguments": info["arguments"]}}]})
                messages.append({"role": "tool", "tool_call_id": cid, "content": str(result)})
            req_id = f"{req_id}-cont"
