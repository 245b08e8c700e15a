"""In-process MI355X engine provider (``LLM_PROVIDER=native``).

``NativeHandler`` exposes the same surface as the reference's ``VLLMHandler``
(``app/core/vllm_handler.py:24-338``: ``check_connection``, ``get_model_info``,
``generate_stream``, ``generate_stream_async``, ``cancel_generation``,
``get_active_requests``) but instead of an HTTP/SSE round trip per token it
submits to the :class:`AsyncEngine` that runs in this process.

Extras the WS server uses:
* ``stream_events`` yields engine ``RequestOutput`` objects (engine token
  counts, time to first token, finish reason);
* per-session token reuse: a follow-up turn is rendered as
  ``previous prompt ids + generated ids + <|eot_id|> + new messages``, so the
  engine's prefix cache matches the whole previous turn even though the
  assistant text was detokenized (re-tokenizing it would not round-trip);
* token-aware history truncation to ``max_model_len - max_tokens``
  (Appendix D Q17): the oldest non-system messages are dropped first.
* history window with hysteresis: once ``ConversationManager`` starts trimming
  to ``max_history_length`` (reference ``conversation_manager.py:34-53``) the
  API history slides by one message per message added, which would change the
  token prefix right after the system block on EVERY turn and defeat the
  prefix cache.  The engine therefore renders a window that is always a suffix
  of the API history (the model never sees more than the reference would) and,
  when the API drops a message the window still holds, cuts the window back to
  ``ENGINE_HISTORY_KEEP`` (fraction of the cap, default 0.5) in one go, so the
  prefix stays stable for the next ~cap/4 turns.  The kept size is jittered per
  session (down by up to ``ENGINE_HISTORY_JITTER`` of the cap, default 0.3), so
  sessions that reach the cap on the same turn cut again on different turns, and
  the window limit itself is lowered per session until its first cut (by up to
  ``ENGINE_HISTORY_LEAD`` of the cap, default 0.15), so a burst of sessions that started together does not
  reach its first cut on the same turn either.
"""
from __future__ import annotations

import asyncio
import hashlib
import logging
import os
import threading
import time
from typing import Any, AsyncIterator, Dict, Iterator, List, Optional

from app.utils.error_handler import ErrorCategory, ErrorSeverity, LLMServiceError

logger = logging.getLogger(__name__)

_ENGINE_LOCK = threading.Lock()
_ENGINES: Dict[str, Any] = {}


def engine_config_from_service(config) -> "Any":
    from fasttalk_llm_microservice_amd.engine.config import EngineConfig

    model = config.resolved_engine_model() if hasattr(config, "resolved_engine_model") else None
    dev = getattr(config, "compute_device", "auto")
    device = "cuda" if dev == "cuda" else ("cpu" if dev in ("cpu", "mps") else "auto")
    cfg = EngineConfig.from_env(model=model)
    cfg.device = device if cfg.device == "auto" else cfg.device
    if getattr(config, "engine_weights", None):
        cfg.weights = config.engine_weights
    if getattr(config, "engine_max_num_seqs", None):
        cfg.max_num_seqs = config.engine_max_num_seqs
    if getattr(config, "engine_max_model_len", None):
        cfg.max_model_len = config.engine_max_model_len
    if getattr(config, "engine_gpu_memory_utilization", None):
        cfg.gpu_memory_utilization = config.engine_gpu_memory_utilization
    if getattr(config, "engine_tp_size", None):
        cfg.tp_size = config.engine_tp_size
    if getattr(config, "engine_dp_size", None):
        cfg.dp_size = config.engine_dp_size
    return cfg


def get_shared_engine(engine_cfg) -> "Any":
    """One engine per (model, weights, device) per process."""
    key = (f"{engine_cfg.model}|{engine_cfg.weights}|{engine_cfg.resolved_device()}|"
           f"{engine_cfg.tp_size}|{engine_cfg.dp_size}|{engine_cfg.separate_process}|"
           f"{engine_cfg.quantization}")
    with _ENGINE_LOCK:
        eng = _ENGINES.get(key)
        if eng is None:
            if engine_cfg.dp_size > 1 or engine_cfg.separate_process:
                from fasttalk_llm_microservice_amd.parallel.dp_router import MultiGPUEngine

                eng = MultiGPUEngine(engine_cfg).start()
            else:
                from fasttalk_llm_microservice_amd.engine.engine import AsyncEngine

                eng = AsyncEngine.from_config(engine_cfg).start()
            _ENGINES[key] = eng
        return eng


def _fingerprint(messages: List[Dict[str, Any]]) -> List[str]:
    out = []
    for m in messages:
        h = hashlib.blake2b(digest_size=12)
        h.update(str(m.get("role", "")).encode())
        h.update(b"\x00")
        h.update(str(m.get("content", "")).encode())
        out.append(h.hexdigest())
    return out


class _SessionTokens:
    __slots__ = ("fps", "head", "prompt_ids", "gen_ids", "reply_fp", "tools_fp", "cut")

    def __init__(self):
        self.fps: List[str] = []          # messages of the engine window (rendered)
        self.head = 0                     # 1 when fps[0] is the system message
        self.prompt_ids: List[int] = []
        self.gen_ids: List[int] = []
        self.reply_fp: Optional[str] = None
        self.tools_fp: str = ""
        self.cut = False                  # the window has been cut at least once


def _tools_fp(tools) -> str:
    if not tools:
        return ""
    import json as _json

    return hashlib.blake2b(_json.dumps(tools, sort_keys=True, default=str).encode(),
                           digest_size=12).hexdigest()


class NativeHandler:
    def __init__(self, config=None, engine=None, model: Optional[str] = None,
                 default_max_tokens: int = 2048):
        self.config = config
        if engine is None:
            engine = get_shared_engine(engine_config_from_service(config))
        self.engine = engine
        inner = getattr(engine, "engine", engine)
        self.tokenizer = inner.tokenizer
        self.template = inner.template
        self.max_model_len = inner.max_model_len
        self.model = model or getattr(inner.model_cfg, "name", "native")
        self.default_max_tokens = default_max_tokens
        self._active: Dict[str, str] = {}      # session/request key -> engine request id
        self._sessions: Dict[str, _SessionTokens] = {}
        self._lock = threading.Lock()
        self._seq = 0
        self.history_cap = int(getattr(config, "max_history_length", 0) or 0)
        self.keep_frac = float(os.environ.get("ENGINE_HISTORY_KEEP", "0.5"))
        self.jitter_frac = float(os.environ.get("ENGINE_HISTORY_JITTER", "0.3"))
        self.lead_frac = float(os.environ.get("ENGINE_HISTORY_LEAD", "0.15"))
        self.warm_cuts = os.environ.get("ENGINE_WARM_CUT_WINDOW", "1").lower() in ("1", "true")
        self.warmups = 0

    # ------------------------------------------------------------------ health / info
    def check_connection(self) -> bool:
        try:
            return bool(self.engine.is_healthy())
        except Exception as e:  # pragma: no cover
            logger.error("engine health check failed: %s", e)
            return False

    def get_model_info(self) -> Dict[str, Any]:
        info = dict(self.engine.model_info())
        return {"models": [self.model], "current_model": self.model, "engine": info}

    def get_active_requests(self) -> Dict[str, Dict[str, Any]]:
        with self._lock:
            return {k: {"engine_request_id": v} for k, v in self._active.items()}

    def forget_session(self, session_id: str):
        with self._lock:
            self._sessions.pop(session_id, None)

    # ------------------------------------------------------------------ prompt building
    def _window_limit(self, session_id: Optional[str]) -> int:
        """Most non-system messages the engine window may hold (0: no count cap):
        what ConversationManager keeps (cap - 1 besides the system prompt), less a
        per-session lead of up to ENGINE_HISTORY_LEAD of it until the window's first
        cut, so sessions that started together (a burst of conversations) do not all
        reach the cap -- and re-prefill a cut window -- on the same turn (that one turn set p99 TTFT: 815 ms at 40
        turns, profiles/bench_40_turns_r02.log)."""
        cap = self.history_cap
        if cap <= 2:
            return 0
        limit = cap - 1
        span = int(self.lead_frac * limit)
        st = self._sessions.get(session_id) if session_id else None
        if span > 0 and session_id and not (st is not None and st.cut):
            h = int(hashlib.blake2b(b"lead:" + str(session_id).encode(), digest_size=4).hexdigest(), 16)
            limit -= h % (span + 1)
        return max(4, limit)

    def _keep(self, limit: int, session_id: Optional[str]) -> int:
        """Messages a cut window keeps: ENGINE_HISTORY_KEEP of the limit, minus a
        per-session jitter of up to ENGINE_HISTORY_JITTER of it, so sessions that
        hit the cap on the same turn cut again on different turns afterwards."""
        keep = self.keep_frac * limit
        span = int(self.jitter_frac * limit)
        if span > 0 and session_id:
            h = int(hashlib.blake2b(str(session_id).encode(), digest_size=4).hexdigest(), 16)
            keep -= h % (span + 1)
        return max(1, min(limit - 1, int(round(keep))))

    def _cut_window(self, msgs: List[Dict[str, Any]], head: int, session_id: Optional[str],
                    at_cap: bool = False):
        """Drops the oldest non-system messages down to the keep size when the
        body exceeds the window limit (or reaches it, ``at_cap``: the API history is
        trimming and no longer continues the previous window); the window starts
        at a user turn."""
        limit = self._window_limit(session_id)
        body = len(msgs) - head
        if not limit or body < limit or (body == limit and not at_cap):
            return msgs
        keep = self._keep(limit, session_id)
        start = len(msgs) - keep
        while start < len(msgs) - 1 and msgs[start].get("role") != "user":
            start += 1
        return msgs[:head] + msgs[start:]

    @staticmethod
    def _find_window(fps: List[str], head: int, prev: List[str], prev_head: int) -> int:
        """Index j such that the previous engine window (system + body) continues
        inside the new history at body offset j with new messages after it; -1 if
        it does not (history edited, or the API dropped part of the window)."""
        if head != prev_head or (head and fps[0] != prev[0]):
            return -1
        body, pbody = fps[head:], prev[prev_head:]
        n = len(pbody)
        for j in range(0, len(body) - n):
            if body[j:j + n] == pbody:
                return j
        return -1

    def build_prompt(self, messages: List[Dict[str, Any]], max_tokens: int,
                     session_id: Optional[str] = None, tools=None, remember: bool = True) -> List[int]:
        """Prompt ids for ``messages``; with ``session_id`` a follow-up turn continues
        the session's previous token stream (so the prefix cache matches it).
        ``remember=False`` continues it without recording this prompt as the
        session's new state: the agent's tool rounds (a guided tool call, the answer
        after the tool result) extend the session's cached prefix, but their
        messages are not part of the API history the next turn continues from."""
        budget = max(16, self.max_model_len - max(1, max_tokens) - 1)
        msgs = list(messages)
        head = 1 if msgs and msgs[0].get("role") == "system" else 0
        fps = _fingerprint(msgs)
        tfp = _tools_fp(tools)
        st = self._sessions.get(session_id) if session_id else None
        ids: Optional[List[int]] = None
        was_cut = False
        if st is not None and st.reply_fp is not None and st.tools_fp == tfp:
            prev = st.fps + [st.reply_fp]
            j = self._find_window(fps, head, prev, st.head)
            n_new = len(msgs) - head - j - (len(prev) - st.head)
            limit = self._window_limit(session_id)
            if j >= 0 and (not limit or len(prev) - st.head + n_new <= limit):
                ids = st.prompt_ids + st.gen_ids + [self.tokenizer.eot_id]
                for m in msgs[len(msgs) - n_new:]:
                    ids += self.template.message_ids(m)
                ids += self.template.generation_prompt()
                msgs = msgs[:head] + msgs[head + j:]
                fps = fps[:head] + fps[head + j:]
                if len(ids) > budget:
                    ids = None
        if ids is None:
            n_before = len(msgs)
            msgs = self._cut_window(msgs, head, session_id, at_cap=st is not None)
            was_cut = len(msgs) < n_before
            ids = self.template.render(msgs, tools=tools)
            if len(ids) > budget:
                # token-aware truncation: drop the oldest non-system messages, down to
                # 3/4 of the budget so the next turns extend the prefix again
                target = max(16, (3 * budget) // 4)
                while len(ids) > target and len(msgs) > head + 1:
                    msgs.pop(head)
                    ids = self.template.render(msgs, tools=tools)
            fps = _fingerprint(msgs)
            if len(ids) > budget:
                ids = ids[-budget:]
        if session_id is not None and remember:
            st = self._sessions.setdefault(session_id, _SessionTokens())
            st.fps, st.head, st.prompt_ids, st.gen_ids, st.reply_fp, st.tools_fp = \
                fps, head, ids, [], None, tfp
            if was_cut:
                st.cut = True
            if self.warm_cuts:
                self._warm_next_cut(messages, msgs, head, session_id, budget, tools)
        return ids

    def _warm_next_cut(self, api_msgs: List[Dict[str, Any]], window: List[Dict[str, Any]],
                       head: int, session_id: str, budget: int, tools=None):
        """When this turn's window plus the next turn's two messages (this reply,
        the next user message) will exceed the window limit, the next turn re-renders
        a cut window (``_cut_window``) and would prefill it on its own critical path
        (TTFT of a ~2-3k token prefill, plus a long step every streaming session
        waits for).  Its prefix -- everything up to this turn's user message -- is
        known now, so it is queued as a background prefill: the engine computes it
        in spare step room while this turn streams, and the cut turn then hits the
        prefix cache for all but its newest two messages."""
        limit = self._window_limit(session_id)
        if not limit or len(window) - head + 2 <= limit:
            return
        keep = self._keep(limit, session_id)
        nxt = list(api_msgs) + [{"role": "assistant", "content": ""}, {"role": "user", "content": ""}]
        start = len(nxt) - keep
        while start < len(nxt) - 1 and nxt[start].get("role") != "user":
            start += 1
        if start >= len(api_msgs):
            return
        ids = self.template.render(nxt[:head] + list(api_msgs[start:]), add_generation_prompt=False,
                                   tools=tools)
        warm = getattr(self.engine, "prefill_background", None)
        if warm is None or len(ids) >= budget:
            return
        warm(ids, session_id=session_id)   # DP: routed to the replica owning the session
        self.warmups += 1

    def _remember_reply(self, session_id: Optional[str], gen_ids: List[int], text: str):
        if not session_id:
            return
        st = self._sessions.get(session_id)
        if st is None:
            return
        st.gen_ids = list(gen_ids)
        st.reply_fp = _fingerprint([{"role": "assistant", "content": text}])[0]

    # ------------------------------------------------------------------ generation
    def _params(self, temperature, max_tokens, top_p, top_k=None, stop=None, seed=None,
                guided=None, ignore_eos=False, min_tokens=0, guided_lazy=False, priority=0):
        from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams

        return SamplingParams(
            temperature=0.7 if temperature is None else float(temperature),
            top_p=1.0 if top_p is None else float(top_p),
            top_k=0 if top_k in (None, -1) else int(top_k),
            max_tokens=int(max_tokens or self.default_max_tokens),
            stop=stop, seed=seed, guided=guided, ignore_eos=ignore_eos, min_tokens=min_tokens,
            guided_lazy=bool(guided_lazy and guided is not None), priority=int(priority))

    async def stream_events(self, messages: List[Dict[str, Any]], temperature: Optional[float] = None,
                            max_tokens: Optional[int] = None, top_p: Optional[float] = None,
                            top_k: Optional[int] = None, stop: Optional[List[str]] = None,
                            request_id: Optional[str] = None, session_id: Optional[str] = None,
                            prompt_ids: Optional[List[int]] = None, tools=None, guided=None,
                            seed: Optional[int] = None, ignore_eos: bool = False,
                            min_tokens: int = 0, prefix_session: Optional[str] = None,
                            assistant_prefix: str = "", guided_lazy: bool = False,
                            priority: int = 0) -> AsyncIterator[Any]:
        """``prefix_session`` (with ``session_id=None``): build the prompt on that
        session's token stream without making this request the session's turn.
        ``assistant_prefix``: text the assistant turn starts with (written into the
        prompt; the output stream holds only what follows it).  ``priority``: > 0
        prefills ahead of waiting prompts of lower priority."""
        mt = int(max_tokens or self.default_max_tokens)
        params = self._params(temperature, mt, top_p, top_k, stop, seed, guided, ignore_eos,
                              min_tokens, guided_lazy, priority)
        if prompt_ids is None:
            if session_id is None and prefix_session is not None:
                prompt_ids = self.build_prompt(messages, mt, prefix_session, tools, remember=False)
            else:
                prompt_ids = self.build_prompt(messages, mt, session_id, tools)
            if assistant_prefix:
                prompt_ids = list(prompt_ids) + self.tokenizer.encode(assistant_prefix)
        key = request_id or session_id or f"native-{time.time_ns()}"
        with self._lock:
            self._seq += 1
            rid = f"{key}#{self._seq}"
            self._active[key] = rid
        gen_ids: List[int] = []
        text_parts: List[str] = []
        try:
            async for out in self.engine.generate(prompt_ids, params, request_id=rid):
                gen_ids.extend(out.token_ids)
                if out.text:
                    text_parts.append(out.text)
                if out.finished and out.finish_reason == "error":
                    raise LLMServiceError(f"engine error: {out.error}", category=ErrorCategory.PROCESSING,
                                          severity=ErrorSeverity.HIGH)
                yield out
            if session_id and not stop and (guided is None or guided_lazy):
                self._remember_reply(session_id, gen_ids, "".join(text_parts))
        finally:
            with self._lock:
                if self._active.get(key) == rid:
                    del self._active[key]

    async def generate_stream_async(self, messages: List[Dict[str, str]], temperature: Optional[float] = None,
                                    max_tokens: Optional[int] = None, top_p: Optional[float] = None,
                                    stop: Optional[List[str]] = None, tools=None,
                                    request_id: Optional[str] = None, top_k: Optional[int] = None,
                                    session_id: Optional[str] = None) -> AsyncIterator[str]:
        async for out in self.stream_events(messages, temperature, max_tokens, top_p, top_k, stop,
                                            request_id, session_id, tools=tools):
            if out.text:
                yield out.text

    def generate_stream(self, messages: List[Dict[str, str]], temperature: Optional[float] = None,
                        max_tokens: Optional[int] = None, top_p: Optional[float] = None,
                        stop: Optional[List[str]] = None, tools=None,
                        request_id: Optional[str] = None, top_k: Optional[int] = None) -> Iterator[str]:
        """Synchronous iterator (drives a private event loop)."""
        loop = asyncio.new_event_loop()
        agen = self.generate_stream_async(messages, temperature, max_tokens, top_p, stop, tools,
                                          request_id, top_k)
        try:
            while True:
                try:
                    yield loop.run_until_complete(agen.__anext__())
                except StopAsyncIteration:
                    break
        finally:
            loop.run_until_complete(agen.aclose())
            loop.close()

    def cancel_generation(self, request_id: str) -> bool:
        with self._lock:
            rid = self._active.get(request_id)
        if rid is None:
            return False
        return bool(self.engine.abort(rid))
