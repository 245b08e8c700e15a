"""Tool-call parsers (E11; Appendix D Q16).

The reference lets vLLM parse tool calls server-side with the ``hermes`` parser
(``docker-compose.vllm.yml:50-51``) although Llama-3.1 natively emits the
``llama3_json`` format.  Both are implemented:

* ``llama3_json``: optional ``<|python_tag|>``, then one or more JSON objects
  ``{"name": ..., "parameters": {...}}`` (``arguments`` accepted too), separated
  by ``;`` or newlines.
* ``hermes``: ``<tool_call>{"name": ..., "arguments": {...}}</tool_call>`` blocks.

``auto`` tries hermes then llama3_json.  ``StreamingToolDetector`` decides from
the first non-blank characters of a stream whether it is a tool call (hold
the text back) or plain speech (stream it immediately).
"""
from __future__ import annotations

import json
import re
import uuid
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

PYTHON_TAG = "<|python_tag|>"
_HERMES = re.compile(r"<tool_call>\s*(.*?)\s*</tool_call>", re.S)


@dataclass
class ToolCall:
    name: str
    arguments: Dict[str, Any]
    id: str = field(default_factory=lambda: f"call_{uuid.uuid4().hex[:12]}")

    def to_openai(self) -> Dict[str, Any]:
        return {"id": self.id, "type": "function",
                "function": {"name": self.name, "arguments": json.dumps(self.arguments)}}


def _coerce(obj: Any) -> Optional[ToolCall]:
    if not isinstance(obj, dict) or not isinstance(obj.get("name"), str):
        return None
    args = obj.get("parameters", obj.get("arguments", {}))
    if isinstance(args, str):
        try:
            args = json.loads(args)
        except json.JSONDecodeError:
            return None
    if not isinstance(args, dict):
        return None
    return ToolCall(obj["name"], args)


def _json_objects(text: str) -> List[Any]:
    """Decode consecutive JSON values separated by whitespace / ';'."""
    dec = json.JSONDecoder()
    out, i = [], 0
    while i < len(text):
        while i < len(text) and text[i] in " \t\r\n;":
            i += 1
        if i >= len(text):
            break
        try:
            obj, j = dec.raw_decode(text, i)
        except json.JSONDecodeError:
            return []
        out.append(obj)
        i = j
    return out


def parse_llama3_json(text: str) -> List[ToolCall]:
    t = text.strip()
    if t.startswith(PYTHON_TAG):
        t = t[len(PYTHON_TAG):].strip()
    if not t.startswith("{"):
        return []
    calls = [_coerce(o) for o in _json_objects(t)]
    return [c for c in calls if c is not None] if calls and all(calls) else []


def parse_hermes(text: str) -> List[ToolCall]:
    calls = []
    for m in _HERMES.finditer(text):
        try:
            c = _coerce(json.loads(m.group(1)))
        except json.JSONDecodeError:
            c = None
        if c is not None:
            calls.append(c)
    return calls


def parse_tool_calls(text: str, fmt: str = "auto") -> Tuple[List[ToolCall], str]:
    """Returns (calls, remaining_content)."""
    if fmt in ("auto", "hermes"):
        calls = parse_hermes(text)
        if calls:
            return calls, _HERMES.sub("", text).strip()
        if fmt == "hermes":
            return [], text
    calls = parse_llama3_json(text)
    if calls:
        return calls, ""
    return [], text


class StreamingToolDetector:
    """Classify a stream as tool call vs speech from its first visible chars."""

    def __init__(self):
        self.buf = ""
        self.mode: Optional[str] = None  # "tool" | "text"

    def feed(self, delta: str) -> Tuple[Optional[str], str]:
        """Returns (mode, text_to_emit_now)."""
        if self.mode == "text":
            return "text", delta
        self.buf += delta
        if self.mode == "tool":
            return "tool", ""
        s = self.buf.lstrip()
        if not s:
            return None, ""
        if s.startswith("{") or s.startswith(PYTHON_TAG) or s.startswith("<tool_call>"):
            self.mode = "tool"
            return "tool", ""
        if PYTHON_TAG.startswith(s) or "<tool_call>".startswith(s):
            return None, ""  # could still become a tag
        self.mode = "text"
        out, self.buf = self.buf, ""
        return "text", out
