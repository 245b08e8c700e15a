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


_NAME_RE = re.compile(r'"name"\s*:\s*"((?:[^"\\]|\\.)*)"')
_ARGS_RE = re.compile(r'"(?:parameters|arguments)"\s*:\s*')


class StreamingToolCallParser:
    """Incremental OpenAI ``delta.tool_calls`` from a llama3_json / hermes stream
    (what vLLM's ``--enable-auto-tool-choice`` streams and the reference's
    ``VLLMWithToolsHandler`` accumulates, ``/root/reference/app/core/vllm_handler.py:389-408``).

    ``feed(delta)`` returns the tool-call deltas that became known: for each call
    first ``{index, id, type, function: {name, arguments: ""}}``, then argument
    fragments ``{index, function: {arguments}}`` as the JSON of the arguments
    object streams in.  The concatenated fragments of a call are exactly the
    arguments' JSON text as the model wrote it.

    ``names``: the request's tool names; an object whose ``"name"`` is not one of
    them is not a call (``self.rejected``, nothing more is emitted) -- e.g. a JSON
    text answer that happens to carry a "name" key."""

    def __init__(self, names=None):
        self.names = set(names) if names is not None else None
        self.rejected = False
        self.buf = ""
        self.obj_start: Optional[int] = None   # offset of the current call's '{'
        self.header_sent = False
        self.args_start: Optional[int] = None  # offset of the arguments value
        self.args_sent = 0                     # chars of the value already emitted
        self.args_end: Optional[int] = None
        self.index = -1
        self.call_id = ""
        self.scan = 0                          # next offset to look for a call at
        self.ncalls = 0

    def _value_end(self, start: int) -> Optional[int]:
        """End offset (exclusive) of the JSON value at ``start`` if complete."""
        s = self.buf
        if start >= len(s):
            return None
        if s[start] not in "{[":
            if s[start] == '"':
                i, esc = start + 1, False
                while i < len(s):
                    c = s[i]
                    if esc:
                        esc = False
                    elif c == "\\":
                        esc = True
                    elif c == '"':
                        return i + 1
                    i += 1
                return None
            m = re.match(r"[^,}\]\s]+", s[start:])
            return start + m.end() if m and start + m.end() < len(s) else None
        depth, i, in_str, esc = 0, start, False, False
        while i < len(s):
            c = s[i]
            if in_str:
                if esc:
                    esc = False
                elif c == "\\":
                    esc = True
                elif c == '"':
                    in_str = False
            elif c == '"':
                in_str = True
            elif c in "{[":
                depth += 1
            elif c in "}]":
                depth -= 1
                if depth == 0:
                    return i + 1
            i += 1
        return None

    def _obj_end(self) -> Optional[int]:
        return self._value_end(self.obj_start)

    def feed(self, delta: str) -> List[Dict[str, Any]]:
        self.buf += delta
        out: List[Dict[str, Any]] = []
        while not self.rejected:
            if self.obj_start is None:
                i = self.buf.find("{", self.scan)
                if i < 0:
                    return out
                self.obj_start = i
                self.header_sent, self.args_start, self.args_sent, self.args_end = False, None, 0, None
            seg = self.buf[self.obj_start:]
            if not self.header_sent:
                m = _NAME_RE.search(seg)
                if m is None:
                    return out
                name = json.loads('"' + m.group(1) + '"')
                if self.names is not None and name not in self.names:
                    self.rejected = True
                    return out
                self.index = self.ncalls
                self.ncalls += 1
                self.call_id = f"call_{uuid.uuid4().hex[:12]}"
                out.append({"index": self.index, "id": self.call_id, "type": "function",
                            "function": {"name": name, "arguments": ""}})
                self.header_sent = True
            if self.args_start is None:
                m = _ARGS_RE.search(seg)
                if m is None:
                    end = self._obj_end()
                    if end is None:
                        return out
                    out.append({"index": self.index, "function": {"arguments": "{}"}})
                    self.obj_start, self.scan = None, end
                    continue
                self.args_start = self.obj_start + m.end()
            while self.args_sent == 0 and self.args_start < len(self.buf) and \
                    self.buf[self.args_start] in " \t\r\n":
                self.args_start += 1  # the key's regex may have matched before the blanks arrived
            if self.args_start >= len(self.buf):
                return out
            end = self.args_end if self.args_end is not None else self._value_end(self.args_start)
            if end is not None:
                self.args_end = end
                raw = self.buf[self.args_start:end]
                if raw.startswith('"'):  # arguments given as a JSON-encoded string
                    try:
                        raw = json.loads(raw)
                    except json.JSONDecodeError:
                        pass
                    frag = raw[self.args_sent:] if self.args_sent == 0 else ""
                else:
                    frag = raw[self.args_sent:]
                if frag:
                    out.append({"index": self.index, "function": {"arguments": frag}})
                self.args_sent = len(raw)
                obj_end = self._obj_end()
                if obj_end is None:
                    return out
                self.obj_start, self.scan = None, obj_end
                continue
            # arguments still streaming: emit what is certainly part of an object value
            avail = self.buf[self.args_start:]
            if avail.startswith("{") or avail.startswith("["):
                frag = avail[self.args_sent:]
                if frag:
                    out.append({"index": self.index, "function": {"arguments": frag}})
                    self.args_sent = len(avail)
            return out
        return out
