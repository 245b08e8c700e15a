"""Remote Ollama backend (``LLM_PROVIDER=ollama``), API of the reference
``app/core/ollama_handler.py`` (``OllamaHandler``: ``check_connection``,
``get_model_info``, ``generate_stream``, ``cancel_generation``,
``get_active_requests``, ``cleanup_stale_requests``, ``close``).

The generator is synchronous (``requests`` NDJSON stream); the WS server drives
it from a worker thread so it never blocks the event loop (Appendix D Q7).
"""
from __future__ import annotations

import codecs
import json
import logging
import time
import uuid
from threading import Lock
from typing import Any, Dict, Generator, List, Optional

import requests

from app.utils.error_handler import ErrorCategory, ErrorSeverity, LLMServiceError

logger = logging.getLogger(__name__)


class OllamaHandler:
    def __init__(self, base_url: str, model: str, keep_alive: str = "5m", timeout: float = 600.0):
        self.base_url = base_url.rstrip("/")
        self.model = model
        self.keep_alive = keep_alive
        self.timeout = timeout
        self.session = requests.Session()
        self._active_requests: Dict[str, Dict[str, Any]] = {}
        self._requests_lock = Lock()
        self._connection_ok = False

    def check_connection(self) -> bool:
        try:
            self.session.get(self.base_url + "/", timeout=5.0).raise_for_status()
            self._connection_ok = True
        except requests.exceptions.RequestException as e:
            logger.error("Failed to connect to Ollama at %s: %s", self.base_url, e)
            self._connection_ok = False
        return self._connection_ok

    def get_model_info(self) -> Dict[str, Any]:
        try:
            r = self.session.post(self.base_url + "/api/show", json={"name": self.model}, timeout=10.0)
            r.raise_for_status()
            return r.json()
        except requests.exceptions.RequestException as e:
            raise LLMServiceError(f"Failed to get model info: {e}", category=ErrorCategory.CONNECTION,
                                  severity=ErrorSeverity.MEDIUM)

    def generate_stream(self, messages: List[Dict[str, str]], temperature: Optional[float] = None,
                        max_tokens: Optional[int] = None, top_p: Optional[float] = None,
                        top_k: Optional[int] = None, stop: Optional[List[str]] = None,
                        request_id: Optional[str] = None) -> Generator[str, None, None]:
        req_id = request_id or f"ollama-{uuid.uuid4()}"
        options = {k: v for k, v in (("temperature", temperature), ("num_predict", max_tokens),
                                     ("top_p", top_p), ("top_k", top_k), ("stop", stop)) if v is not None}
        payload = {"model": self.model, "messages": messages, "stream": True, "options": options,
                   "keep_alive": self.keep_alive}
        resp = None
        try:
            resp = self.session.post(self.base_url + "/api/chat", json=payload, stream=True,
                                     timeout=(10.0, self.timeout))
            resp.raise_for_status()
            with self._requests_lock:
                self._active_requests[req_id] = {"stream": resp, "start_time": time.time()}
            buf = ""
            # incremental: a multi-byte UTF-8 character split across HTTP chunks is
            # completed by the next chunk instead of becoming U+FFFD
            dec = codecs.getincrementaldecoder("utf-8")(errors="replace")
            for raw in resp.iter_content(chunk_size=None):
                with self._requests_lock:
                    if req_id not in self._active_requests:
                        break
                if not raw:
                    continue
                buf += dec.decode(raw)
                done = False
                while "\n" in buf:
                    line, buf = buf.split("\n", 1)
                    if not line.strip():
                        continue
                    try:
                        obj = json.loads(line)
                    except json.JSONDecodeError:
                        continue
                    if obj.get("error"):
                        raise LLMServiceError(f"Ollama stream error: {obj['error']}",
                                              category=ErrorCategory.PROCESSING,
                                              severity=ErrorSeverity.HIGH)
                    text = (obj.get("message") or {}).get("content")
                    if text:
                        yield text
                    if obj.get("done"):
                        done = True
                        break
                if done:
                    break
        except LLMServiceError:
            raise
        except requests.exceptions.ConnectionError as e:
            raise LLMServiceError(f"Connection error during generation: {e}",
                                  category=ErrorCategory.CONNECTION, severity=ErrorSeverity.HIGH)
        except requests.exceptions.Timeout as e:
            raise LLMServiceError(f"Timeout during generation: {e}", category=ErrorCategory.TIMEOUT,
                                  severity=ErrorSeverity.MEDIUM, retry_after=30.0)
        except requests.exceptions.ChunkedEncodingError as e:
            with self._requests_lock:
                cancelled = req_id not in self._active_requests
            if not cancelled:
                raise LLMServiceError(f"Stream encoding error: {e}", category=ErrorCategory.CONNECTION,
                                      severity=ErrorSeverity.HIGH)
        except requests.exceptions.HTTPError as e:
            raise LLMServiceError(f"HTTP error during generation: {e}",
                                  category=ErrorCategory.PROCESSING, severity=ErrorSeverity.HIGH)
        except Exception as e:
            raise LLMServiceError(f"Unexpected error during generation: {e}",
                                  category=ErrorCategory.SYSTEM, severity=ErrorSeverity.CRITICAL)
        finally:
            with self._requests_lock:
                self._active_requests.pop(req_id, None)
            if resp is not None:
                try:
                    resp.close()
                except Exception:
                    pass

    def _cancel_locked(self, req_id: str) -> bool:
        info = self._active_requests.pop(req_id, None)
        if info is None:
            return False
        try:
            info["stream"].close()
        except Exception:
            pass
        return True

    def cancel_generation(self, request_id: Optional[str] = None) -> bool:
        with self._requests_lock:
            if request_id is None:
                ids = list(self._active_requests)
                return any([self._cancel_locked(r) for r in ids])
            return self._cancel_locked(request_id)

    def get_active_requests(self) -> List[str]:
        with self._requests_lock:
            return list(self._active_requests)

    def cleanup_stale_requests(self, timeout_seconds: int = 300) -> int:
        now = time.time()
        with self._requests_lock:
            stale = [r for r, i in self._active_requests.items() if now - i["start_time"] > timeout_seconds]
        return sum(1 for r in stale if self.cancel_generation(r))

    def close(self):
        self.cancel_generation(None)
        self.session.close()
