"""Llama-3 chat template rendered straight to token ids (E2).

The reference hands OpenAI-shaped ``messages`` (``conversation_manager.py:36,
125-126``; tool messages at ``vllm_handler.py:425-440``) to vLLM, which applies
the model's chat template.  We render the Llama-3.1 header format ourselves:

    <|begin_of_text|>
    <|start_header_id|>{role}<|end_header_id|>\\n\\n{content}<|eot_id|>  (per message)
    <|start_header_id|>assistant<|end_header_id|>\\n\\n                  (generation prompt)

Every message is encoded independently, so the ids of a conversation are a
strict prefix of the ids of the same conversation one turn later -- the
property the engine's prefix cache (multi-turn KV reuse) depends on.
Tool definitions are rendered into the system message in the Llama-3.1 JSON
function-calling style; assistant tool calls are rendered as
``{"name": ..., "parameters": ...}`` and tool results use the ``ipython`` role.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional, Sequence

from .tokenizer import Tokenizer

TOOL_INSTRUCTIONS = (
    "You have access to the following functions. To call a function, respond only with a JSON "
    "object of the form {\"name\": function name, \"parameters\": dictionary of argument name and "
    "its value}. Do not use variables. If no function is needed, answer the user directly.\n\n")


def render_tools(tools: Sequence[Dict[str, Any]]) -> str:
    parts = []
    for t in tools:
        fn = t.get("function", t)
        parts.append(json.dumps({"type": "function", "function": fn}, separators=(", ", ": ")))
    return TOOL_INSTRUCTIONS + "\n\n".join(parts)


def _content_text(m: Dict[str, Any]) -> str:
    c = m.get("content")
    if c is None:
        c = ""
    if isinstance(c, list):  # OpenAI content parts
        c = "".join(p.get("text", "") for p in c if isinstance(p, dict))
    if m.get("tool_calls"):
        calls = []
        for tc in m["tool_calls"]:
            fn = tc.get("function", tc)
            args = fn.get("arguments", fn.get("parameters", {}))
            if isinstance(args, str):
                try:
                    args = json.loads(args)
                except json.JSONDecodeError:
                    pass
            calls.append(json.dumps({"name": fn.get("name"), "parameters": args}))
        c = (c + "\n" if c else "") + "\n".join(calls)
    return str(c)


class ChatTemplate:
    # rendered messages kept (role, text) -> ids: a conversation re-renders the same
    # history messages at every window cut and for the cut-window warm-up, and each
    # encode runs on the service's event loop (~0.25 ms per message)
    MSG_CACHE = 16384

    def __init__(self, tokenizer: Tokenizer):
        self.tok = tokenizer
        self._hdr_cache: Dict[str, List[int]] = {}
        self._msg_cache: Dict[tuple, List[int]] = {}

    def _header(self, role: str) -> List[int]:
        h = self._hdr_cache.get(role)
        if h is None:
            h = [self.tok.start_header_id] + self.tok.encode(role) + [self.tok.end_header_id] + \
                self.tok.encode("\n\n")
            self._hdr_cache[role] = h
        return h

    def message_ids(self, m: Dict[str, Any]) -> List[int]:
        role = m.get("role", "user")
        if role == "tool":
            role = "ipython"
        text = _content_text(m)
        key = (role, text)
        ids = self._msg_cache.get(key)
        if ids is None:
            ids = self._header(role) + self.tok.encode(text) + [self.tok.eot_id]
            while len(self._msg_cache) >= self.MSG_CACHE:   # FIFO: drop the oldest entries
                try:
                    self._msg_cache.pop(next(iter(self._msg_cache)))
                except (RuntimeError, KeyError, StopIteration):   # a concurrent render
                    self._msg_cache.clear()
            self._msg_cache[key] = ids
        return list(ids)

    def remember_assistant(self, ids: Sequence[int]) -> None:
        """Token-exact history: the ids an assistant turn was GENERATED as, filed under the
        text they decode to, so the next turn renders that message with the same ids and
        the engine's prefix cache covers the whole reply.  This is the path of stateless
        clients (the OpenAI facade, /v1/chat/completions, and any render after a history
        window cut) that send the reply back as text; a WS session continues from its
        own token state (NativeHandler).  Re-encoding a generated reply
        rarely reproduces its ids (a sampled sequence is seldom the tokenizer's own
        segmentation of its text: 40% of a random 128-token reply survived a round trip
        on the synthetic tokenizer), and every token after the first mismatch is
        prefilled again.  A message stored with any other text (stop-string cuts,
        post-processing) simply misses the entry and is encoded as before."""
        ids = list(ids)
        if not ids or any(self.tok.is_special(t) for t in ids):
            return
        key = ("assistant", self.tok.decode(ids))
        while len(self._msg_cache) >= self.MSG_CACHE:
            try:
                self._msg_cache.pop(next(iter(self._msg_cache)))
            except (RuntimeError, KeyError, StopIteration):
                self._msg_cache.clear()
        self._msg_cache[key] = self._header("assistant") + ids + [self.tok.eot_id]

    def render(self, messages: Sequence[Dict[str, Any]], add_generation_prompt: bool = True,
               tools: Optional[Sequence[Dict[str, Any]]] = None) -> List[int]:
        msgs = list(messages)
        if tools:
            if msgs and msgs[0].get("role") == "system":
                msgs[0] = dict(msgs[0], content=render_tools(tools) + "\n\n" + _content_text(msgs[0]))
            else:
                msgs.insert(0, {"role": "system", "content": render_tools(tools)})
        ids = [self.tok.bos_id]
        for m in msgs:
            ids += self.message_ids(m)
        if add_generation_prompt:
            ids += self.generation_prompt()
        return ids

    def generation_prompt(self) -> List[int]:
        return list(self._header("assistant"))

    def render_text(self, messages, add_generation_prompt=True, tools=None) -> str:
        return self.tok.decode(self.render(messages, add_generation_prompt, tools),
                               skip_special_tokens=False)
