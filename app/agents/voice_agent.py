"""Voice agent with tool calling (E18) -- API of the reference
``app/agents/voice_agent.py`` (``ConversationContext``, ``AgentConfig``,
``VoiceAgent.generate_stream / generate / update_config / check_connection /
get_model_info``).

pydantic-ai is not installable offline, so the agent loop is native:
  render messages + tool schemas (Llama-3.1 JSON tool calling) -> stream from the
  backend -> a StreamingToolDetector decides from the first visible characters
  whether the reply is a tool call (held back) or speech (streamed at once) ->
  tool calls are parsed (llama3_json / hermes), executed, appended as assistant
  tool-call + ``ipython`` result messages, and the model is re-prompted, up to
  ``max_tool_rounds``.

Differences from the reference (Appendix D): multi-turn history is passed as
real chat messages to the native engine (prefix-cache friendly, Q18; the
reference's flattened "Previous conversation:" prompt is still available as
``_build_prompt_with_history`` and is used for remote backends, which run the
same tool loop over the OpenAI API: schemas sent, streamed ``tool_calls`` deltas
assembled, tools run here, results re-prompted -- the reference's PydanticAI path);
``temperature
= 0`` means greedy (Q5); with ``guided_tool_calls`` (or ``tool_choice=
"required"``) the tool call is decoded under a JSON-schema token FSM, so even
random-init weights produce a valid call (BASELINE config 5).
"""
from __future__ import annotations

import json
import logging
import os
import re
from dataclasses import dataclass, field
from datetime import datetime
from typing import Any, AsyncGenerator, Dict, List, Optional

from pydantic import BaseModel

from app.agents.tools import Tool, make_search_tool, make_session_tool, make_time_tool

logger = logging.getLogger(__name__)

_TOOL_HINTS = re.compile(r"\b(search|look up|lookup|news|weather|latest|current|today|time|date|"
                         r"session|google|find)\b", re.I)
# hint words that name one tool: a message whose hints all point at one tool forces
# that tool (its call's fixed head is then prefilled); mixed or ambiguous hints
# ("current", "today") leave the choice among all tools to the model
_HINT_TOOLS = ((re.compile(r"\b(search|look up|lookup|news|weather|latest|google|find)\b", re.I),
                "duckduckgo_search"),
               (re.compile(r"\b(time|date)\b", re.I), "get_current_time"),
               (re.compile(r"\bsession\b", re.I), "get_session_info"))


@dataclass
class ConversationContext:
    user_id: str
    session_id: str
    conversation_history: List[Dict[str, str]] = field(default_factory=list)
    language: str = "en"
    created_at: datetime = field(default_factory=datetime.now)
    metadata: Dict[str, Any] = field(default_factory=dict)

    def add_message(self, role: str, content: str):
        self.conversation_history.append({"role": role, "content": content,
                                          "timestamp": datetime.now().isoformat()})

    def get_recent_messages(self, limit: int = 10) -> List[Dict[str, str]]:
        return self.conversation_history[-limit:]


class AgentConfig(BaseModel):
    vllm_base_url: str = "http://vllm:8000/v1"
    vllm_model: str = "hugging-quants/Meta-Llama-3.1-8B-Instruct-AWQ-INT4"
    vllm_api_key: str = "not-needed"
    temperature: float = 0.7
    max_tokens: int = 2048
    top_p: float = 0.9
    enable_web_search: bool = True
    enable_tools: bool = True
    duckduckgo_rate_limit: float = 1.0
    system_prompt: str = ("You are a helpful voice assistant for FastTalk. Keep your responses concise "
                          "and conversational, suitable for speech synthesis. When asked about current "
                          "events or facts you're unsure about, use web search. Avoid long lists or "
                          "complex formatting - speak naturally as if in a conversation.")
    guided_tool_calls: bool = False
    max_tool_rounds: int = 3
    # one forced tool: write its call's fixed head into the prompt (AGENT_PREFILL_TOOL_HEAD)
    prefill_tool_head: bool = True
    # the model decides (AGENT_MODEL_TOOL_CHOICE): every round offers the tool-call grammar
    # lazily -- bound only if the model's first token opens a call, free text otherwise --
    # so a real checkpoint picks tools itself and its calls are always valid JSON (the
    # keyword router behind guided_tool_calls exists for random weights)
    model_tool_choice: bool = False
    # scheduling priority of a tool round's follow-up request (AGENT_TOOL_ROUND_PRIORITY,
    # opt-in): > 0 prefills the re-prompt ahead of waiting prompts that have not started
    # (engine Scheduler.add); 0 queues it in arrival order like any new turn.  Measured
    # neutral at config 5 with the mixed chain (profiles/ab_tool_round_priority_r05.log)
    tool_round_priority: int = 0


@dataclass(slots=True)
class AgentEvent:
    text: str = ""
    num_tokens: int = 0
    finish_reason: Optional[str] = None
    prompt_tokens: int = 0
    cached_tokens: int = 0
    tool_call: Optional[Dict[str, Any]] = None
    tool_result: Optional[str] = None
    engine_ttft_s: Optional[float] = None   # request arrival -> first token inside the engine


class VoiceAgent:
    def __init__(self, config: Optional[AgentConfig] = None, backend=None):
        self.config = config or self._load_config_from_env()
        self.backend = backend
        self._tools: Optional[Dict[str, Tool]] = None
        self._custom: Dict[str, Tool] = {}
        self._active: Dict[str, str] = {}

    def _load_config_from_env(self) -> AgentConfig:
        e = os.getenv
        return AgentConfig(
            vllm_base_url=e("VLLM_BASE_URL", "http://vllm:8000/v1"),
            vllm_model=e("VLLM_MODEL", AgentConfig().vllm_model),
            vllm_api_key=e("VLLM_API_KEY", "not-needed"),
            temperature=float(e("DEFAULT_TEMPERATURE", "0.7")),
            max_tokens=int(e("DEFAULT_MAX_TOKENS", "2048")),
            top_p=float(e("DEFAULT_TOP_P", "0.9")),
            enable_web_search=e("ENABLE_WEB_SEARCH", "true").lower() == "true",
            enable_tools=e("ENABLE_TOOLS", "true").lower() == "true",
            duckduckgo_rate_limit=float(e("DUCKDUCKGO_RATE_LIMIT", "1.0")),
            system_prompt=e("SYSTEM_PROMPT", AgentConfig().system_prompt),
            guided_tool_calls=e("AGENT_GUIDED_TOOL_CALLS", "false").lower() == "true",
            prefill_tool_head=e("AGENT_PREFILL_TOOL_HEAD", "true").lower() == "true",
            model_tool_choice=e("AGENT_MODEL_TOOL_CHOICE", "false").lower() == "true",
            tool_round_priority=int(e("AGENT_TOOL_ROUND_PRIORITY", "0")),
        )

    # ------------------------------------------------------------------ backend
    def _get_backend(self):
        if self.backend is None:
            from app.core.vllm_handler import VLLMHandler

            self.backend = VLLMHandler(self.config.vllm_base_url, self.config.vllm_model,
                                       self.config.vllm_api_key)
        return self.backend

    @property
    def is_native(self) -> bool:
        return hasattr(self._get_backend(), "stream_events")

    # ------------------------------------------------------------------ tools
    def tool(self, fn=None, *, name: Optional[str] = None, description: Optional[str] = None,
             parameters: Optional[Dict[str, Any]] = None):
        """Decorator registering a custom tool ``fn(ctx, **kwargs)`` (sync or async)."""
        def deco(f):
            t = Tool(name or f.__name__, description or (f.__doc__ or "").strip(),
                     parameters or {"type": "object", "properties": {}}, f)
            self._custom[t.name] = t
            self._tools = None
            return f
        return deco(fn) if fn is not None else deco

    def tools(self) -> Dict[str, Tool]:
        if self._tools is None:
            tools: Dict[str, Tool] = {}
            if self.config.enable_tools:
                if self.config.enable_web_search:
                    t = make_search_tool(self.config.duckduckgo_rate_limit)
                    tools[t.name] = t
                for t in (make_time_tool(), make_session_tool()):
                    tools[t.name] = t
                tools.update(self._custom)
            self._tools = tools
        return self._tools

    def tool_schemas(self) -> List[Dict[str, Any]]:
        return [t.schema() for t in self.tools().values()]

    # ------------------------------------------------------------------ prompts
    def _build_prompt_with_history(self, user_message: str, context: ConversationContext) -> str:
        """Reference prompt format (last 10 messages flattened), kept for API fidelity."""
        recent = context.get_recent_messages(limit=10)
        if not recent:
            return user_message
        hist = "\n".join(f"{m['role'].capitalize()}: {m['content']}" for m in recent)
        return f"Previous conversation:\n{hist}\n\nCurrent message from user: {user_message}"

    def _messages(self, user_message: str, context: ConversationContext) -> List[Dict[str, Any]]:
        hist = [dict(role=m["role"], content=m["content"]) for m in context.conversation_history]
        if hist and hist[0]["role"] == "system":
            system, hist = hist[0]["content"], hist[1:]
        else:
            system = self.config.system_prompt
        return [{"role": "system", "content": system}] + hist + [{"role": "user", "content": user_message}]

    def _wants_tool(self, user_message: str, tool_choice: Optional[str]) -> Optional[str]:
        if not self.tools():
            return None
        if tool_choice in ("required",) or (tool_choice and tool_choice in self.tools()):
            return tool_choice
        if tool_choice in (None, "auto") and self.config.guided_tool_calls and \
                _TOOL_HINTS.search(user_message or ""):
            msg = user_message or ""
            named = {name for rx, name in _HINT_TOOLS if rx.search(msg)}
            ambiguous = re.search(r"\b(current|today)\b", msg, re.I) is not None
            if len(named) == 1 and not ambiguous and next(iter(named)) in self.tools():
                return next(iter(named))
            return "required"
        return None

    # ------------------------------------------------------------------ generation
    async def generate_events(self, user_message: str, context: ConversationContext,
                              temperature: Optional[float] = None, max_tokens: Optional[int] = None,
                              top_p: Optional[float] = None, top_k: Optional[int] = None,
                              stop=None, seed: Optional[int] = None, tool_choice: Optional[str] = None,
                              ignore_eos: bool = False, min_tokens: int = 0
                              ) -> AsyncGenerator[AgentEvent, None]:
        temp = self.config.temperature if temperature is None else temperature
        mt = self.config.max_tokens if max_tokens is None else max_tokens
        tp = self.config.top_p if top_p is None else top_p
        backend = self._get_backend()
        if not self.is_native:
            async for ev in self._remote_events(backend, user_message, context, temp, mt, tp, top_k,
                                                stop, seed, tool_choice, ignore_eos, min_tokens):
                yield ev
            return

        from fasttalk_llm_microservice_amd.engine.guided import GuidedSpec
        from fasttalk_llm_microservice_amd.engine.tool_parser import StreamingToolDetector, parse_tool_calls

        messages = self._messages(user_message, context)
        schemas = self.tool_schemas()
        force = self._wants_tool(user_message, tool_choice)
        tools_by_name = self.tools()
        for rnd in range(self.config.max_tool_rounds + 1):
            guided = None
            lazy = False
            head = ""
            if (not force or rnd > 0) and schemas and self.config.model_tool_choice and \
                    rnd < self.config.max_tool_rounds:
                guided, lazy = GuidedSpec.tool_call(schemas), True
            if force and rnd == 0:
                pick = [s for s in schemas if force == "required" or s["function"]["name"] == force]
                if len(pick) == 1 and self.config.prefill_tool_head:
                    # one possible tool: its call's fixed head goes into the prompt
                    # (one prefill instead of a decode step per token of it)
                    head, guided = GuidedSpec.tool_call_tail(pick[0])
                else:
                    guided = GuidedSpec.tool_call(pick or schemas)
            det = StreamingToolDetector() if (schemas and rnd < self.config.max_tool_rounds) else None
            if det is not None and head:
                det.feed(head)
            held: List[str] = []
            held_tokens = 0
            finish = None
            sid = context.session_id
            # a guided call is a finite JSON language: give it room to finish even
            # when the spoken-reply budget is small
            round_mt = max(mt, 256) if guided is not None and not lazy else mt
            async for out in backend.stream_events(
                    messages, temperature=temp, max_tokens=round_mt, top_p=tp, top_k=top_k, stop=stop,
                    request_id=sid, session_id=sid if (rnd == 0 and (guided is None or lazy)) else None,
                    prefix_session=sid, assistant_prefix=head, tools=schemas or None, guided=guided,
                    seed=seed, guided_lazy=lazy,
                    ignore_eos=ignore_eos and (guided is None or lazy), min_tokens=min_tokens,
                    priority=self.config.tool_round_priority if rnd > 0 else 0):
                if out.finished:
                    finish = out.finish_reason
                n = len(out.token_ids)
                if det is None:
                    if out.text or n:
                        yield AgentEvent(text=out.text, num_tokens=n, engine_ttft_s=out.ttft_s,
                                         prompt_tokens=out.num_prompt_tokens,
                                         cached_tokens=out.num_cached_tokens)
                    continue
                mode, emit = det.feed(out.text)
                if mode == "text":
                    if held_tokens:
                        n += held_tokens
                        held_tokens = 0
                    if emit or n:
                        yield AgentEvent(text=emit, num_tokens=n, prompt_tokens=out.num_prompt_tokens,
                                         engine_ttft_s=out.ttft_s,
                                         cached_tokens=out.num_cached_tokens)
                else:
                    held.append(out.text)
                    held_tokens += n
            if det is not None and det.mode != "text":
                text = det.buf
                calls, rest = parse_tool_calls(text)
                calls = [c for c in calls if c.name in tools_by_name]
                if calls and finish != "abort":
                    assistant = {"role": "assistant", "content": "",
                                 "tool_calls": [c.to_openai() for c in calls]}
                    messages.append(assistant)
                    for c in calls:
                        try:
                            result = await tools_by_name[c.name](context, **c.arguments)
                        except TypeError as e:
                            result = f"[Error executing tool: {e}]"
                        except Exception as e:
                            result = f"[Error executing tool: {e}]"
                        yield AgentEvent(num_tokens=held_tokens, tool_call={"name": c.name,
                                                                            "arguments": c.arguments},
                                         tool_result=result)
                        held_tokens = 0
                        messages.append({"role": "tool", "tool_call_id": c.id, "content": result})
                    continue
                # not a valid call: speak what was held back
                if text or held_tokens:
                    yield AgentEvent(text=text, num_tokens=held_tokens)
            yield AgentEvent(finish_reason=finish or "stop")
            return
        yield AgentEvent(finish_reason="length")

    async def _remote_events(self, backend, user_message: str, context: ConversationContext,
                             temp, mt, tp, top_k, stop, seed, tool_choice, ignore_eos, min_tokens
                             ) -> AsyncGenerator[AgentEvent, None]:
        """The reference's default path (PydanticAI over the vLLM OpenAI API,
        ``/root/reference/app/agents/voice_agent.py:141-164,219-229``): the flattened
        history prompt, the tool schemas sent with every request (the server parses
        calls: ``--enable-auto-tool-choice``), streamed ``tool_calls`` deltas
        assembled, the tools run here, their results appended as ``tool`` messages
        and the model re-prompted until it answers in text."""
        prompt = self._build_prompt_with_history(user_message, context)
        messages: List[Dict[str, Any]] = [{"role": "system", "content": self.config.system_prompt},
                                          {"role": "user", "content": prompt}]
        schemas = self.tool_schemas()
        tools_by_name = self.tools()
        force = self._wants_tool(user_message, tool_choice)
        extra = {"top_k": top_k, "seed": seed, "ignore_eos": True if ignore_eos else None,
                 "min_tokens": min_tokens or None}
        chat = getattr(backend, "stream_chat_async", None)
        for rnd in range(self.config.max_tool_rounds + 1):
            offer = bool(schemas) and rnd < self.config.max_tool_rounds and chat is not None
            choice = None
            if offer:
                if force == "required" and rnd == 0:
                    choice = "required"
                elif force and rnd == 0:
                    choice = {"type": "function", "function": {"name": force}}
                else:
                    choice = "auto"
            if chat is None:   # a backend without the chat/tool API: text only
                async for text in backend.generate_stream_async(
                        messages=messages, temperature=temp, max_tokens=mt, top_p=tp,
                        request_id=context.session_id):
                    yield AgentEvent(text=text, num_tokens=1)
                yield AgentEvent(finish_reason="stop")
                return
            calls: List[Dict[str, Any]] = []
            finish = "stop"
            forced = choice not in (None, "auto")
            # a forced call is a finite JSON language: room to finish it, and no ignore_eos
            rx = dict(extra, ignore_eos=None) if forced else extra
            async for ev in chat(messages, temperature=temp, max_tokens=max(mt, 256) if forced else mt,
                                 top_p=tp, stop=stop, tools=schemas if offer else None,
                                 tool_choice=choice, request_id=context.session_id, extra=rx):
                if ev["type"] == "text":
                    yield AgentEvent(text=ev["text"], num_tokens=1)
                elif ev["type"] == "tool_calls":
                    calls = [c for c in ev["calls"] if c.get("name") in tools_by_name]
                else:
                    finish = ev["reason"]
            if not calls or finish == "abort":
                yield AgentEvent(finish_reason=finish)
                return
            messages.append({"role": "assistant", "content": "", "tool_calls": [
                {"id": c["id"], "type": "function",
                 "function": {"name": c["name"], "arguments": c["arguments"] or "{}"}} for c in calls]})
            for c in calls:
                try:
                    args = json.loads(c["arguments"] or "{}")
                    if not isinstance(args, dict):
                        raise ValueError("tool arguments must be a JSON object")
                    result = await tools_by_name[c["name"]](context, **args)
                except Exception as e:   # surfaced to the model, like the reference's handler
                    args = {}
                    result = f"[Error executing tool: {e}]"
                yield AgentEvent(tool_call={"name": c["name"], "arguments": args}, tool_result=result)
                messages.append({"role": "tool", "tool_call_id": c["id"], "content": str(result)})
        yield AgentEvent(finish_reason="length")

    async def generate_stream(self, user_message: str, context: ConversationContext,
                              temperature: Optional[float] = None,
                              max_tokens: Optional[int] = None) -> AsyncGenerator[str, None]:
        async for ev in self.generate_events(user_message, context, temperature, max_tokens):
            if ev.text:
                yield ev.text

    async def generate(self, user_message: str, context: ConversationContext,
                       temperature: Optional[float] = None, max_tokens: Optional[int] = None) -> str:
        return "".join([t async for t in self.generate_stream(user_message, context, temperature,
                                                             max_tokens)])

    def cancel(self, session_id: str) -> bool:
        be = self._get_backend()
        return bool(getattr(be, "cancel_generation", lambda _s: False)(session_id))

    def update_config(self, **kwargs):
        for k, v in kwargs.items():
            if hasattr(self.config, k):
                setattr(self.config, k, v)
        self._tools = None

    def check_connection(self) -> bool:
        try:
            return bool(self._get_backend().check_connection())
        except Exception as e:
            logger.error("agent backend check failed: %s", e)
            return False

    def get_model_info(self) -> Dict[str, Any]:
        be = self._get_backend()
        model = getattr(be, "model", self.config.vllm_model)
        return {
            "model": model,
            "base_url": "in-process" if self.is_native else self.config.vllm_base_url,
            "temperature": self.config.temperature,
            "max_tokens": self.config.max_tokens,
            "web_search_enabled": self.config.enable_web_search,
            "tools_enabled": self.config.enable_tools,
            "tools": list(self.tools()),
        }
