"""JSON-schema constrained decoding (E19): lowers a (subset of) JSON Schema into
the regular grammar AST consumed by the C++ token FSM (csrc/runtime/json_fsm.cpp).

Supported: object (properties emitted in declaration order, required ones --
or all when none are required), string (bounded length, ``enum``), integer,
number, boolean, null, array (bounded items), ``anyOf``/``oneOf`` of those.
Formatting is canonical (``", "`` and ``": "`` separators, no free whitespace),
which keeps the language finite: every path reaches an accepting state, so a
constrained request always terminates with valid JSON.

``tool_call_spec(tools)`` builds the Llama-3.1 JSON tool-call shape
``{"name": <one of the tool names>, "parameters": <that tool's schema>}``.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional, Sequence

MAX_STR = 48
MAX_ITEMS = 4
_STR_EXCLUDE = b'"\\' + bytes(range(0, 32))


def lit(s: str) -> Dict[str, Any]:
    return {"t": "lit", "s": s.encode("utf-8")}


def seq(*c) -> Dict[str, Any]:
    return {"t": "seq", "c": [x for x in c if x is not None]}


def alt(*c) -> Dict[str, Any]:
    return {"t": "alt", "c": list(c)}


def chars(allowed: bytes, neg: bool, lo: int, hi: int) -> Dict[str, Any]:
    return {"t": "chars", "set": allowed, "neg": neg, "min": lo, "max": hi}


def rep(item, lo: int, hi: int, sep=None) -> Dict[str, Any]:
    d = {"t": "rep", "c": item, "min": lo, "max": hi}
    if sep is not None:
        d["sep"] = sep
    return d


_DIG = b"0123456789"


def _integer():
    return seq(alt(lit(""), lit("-")), alt(lit("0"), seq(chars(b"123456789", False, 1, 1),
                                                             chars(_DIG, False, 0, 8))))


def schema_ast(schema: Optional[Dict[str, Any]], depth: int = 0) -> Dict[str, Any]:
    if not schema:
        return lit("{}") if depth == 0 else alt(lit("null"), lit("true"), lit("false"), lit("0"),
                                                 seq(lit('"'), chars(_STR_EXCLUDE, True, 0, MAX_STR), lit('"')))
    if "enum" in schema:
        return alt(*[lit(json.dumps(v)) for v in schema["enum"]])
    if "const" in schema:
        return lit(json.dumps(schema["const"]))
    for key in ("anyOf", "oneOf"):
        if key in schema:
            return alt(*[schema_ast(s, depth + 1) for s in schema[key]])
    t = schema.get("type", "object")
    if isinstance(t, list):
        return alt(*[schema_ast(dict(schema, type=x), depth + 1) for x in t])
    if t == "string":
        hi = min(int(schema.get("maxLength", MAX_STR)), MAX_STR)
        lo = min(int(schema.get("minLength", 1)), hi)
        return seq(lit('"'), chars(_STR_EXCLUDE, True, lo, hi), lit('"'))
    if t == "integer":
        return _integer()
    if t == "number":
        return seq(_integer(), alt(lit(""), seq(lit("."), chars(_DIG, False, 1, 6))))
    if t == "boolean":
        return alt(lit("true"), lit("false"))
    if t == "null":
        return lit("null")
    if t == "array":
        item = schema_ast(schema.get("items", {"type": "string"}), depth + 1)
        hi = min(int(schema.get("maxItems", MAX_ITEMS)), MAX_ITEMS)
        lo = min(int(schema.get("minItems", 0)), hi)
        return seq(lit("["), rep(item, lo, hi, lit(", ")), lit("]"))
    # object
    props = schema.get("properties", {}) or {}
    req = schema.get("required") or list(props.keys())
    names = [n for n in props if n in req]
    if not names:
        return lit("{}")
    parts: List[Any] = [lit("{")]
    for i, n in enumerate(names):
        if i:
            parts.append(lit(", "))
        parts.append(lit(json.dumps(n) + ": "))
        parts.append(schema_ast(props[n], depth + 1))
    parts.append(lit("}"))
    return seq(*parts)


def tool_call_ast(tools: Sequence[Dict[str, Any]]) -> Dict[str, Any]:
    branches = []
    for t in tools:
        fn = t.get("function", t)
        branches.append(seq(lit(json.dumps(fn["name"])), lit(', "parameters": '),
                            schema_ast(fn.get("parameters") or {"type": "object"}, 1)))
    return seq(lit('{"name": '), alt(*branches), lit("}"))


def _peel_literal(ast: Dict[str, Any]):
    """(fixed leading bytes, the rest of the grammar or None when nothing is left):
    the literal run a grammar must start with, e.g. ``{"query": "`` of an object
    whose first property is a string."""
    if ast["t"] == "lit":
        return ast["s"], None
    if ast["t"] == "seq":
        acc = b""
        kids = ast["c"]
        for i, k in enumerate(kids):
            p, r = _peel_literal(k)
            acc += p
            if r is not None:
                return acc, seq(r, *kids[i + 1:])
        return acc, None
    return b"", ast


class GuidedSpec:
    """Attach to ``SamplingParams.guided``; the engine compiles it lazily."""

    _cache: Dict[str, Any] = {}

    def __init__(self, ast: Dict[str, Any]):
        self.ast = ast
        self.key = json.dumps(ast, sort_keys=True, default=lambda b: b.hex())

    def grammar(self, engine) -> Any:
        from ..runtime import rt

        k = (id(engine), self.key)
        g = GuidedSpec._cache.get(k)
        if g is None:
            eos = [engine.tokenizer.eot_id, engine.tokenizer.eom_id]
            g = rt().Grammar(self.ast, engine.token_trie(), eos)
            GuidedSpec._cache[k] = g
        return g

    @classmethod
    def json_schema(cls, schema: Dict[str, Any]) -> "GuidedSpec":
        return cls(schema_ast(schema))

    @classmethod
    def tool_call(cls, tools: Sequence[Dict[str, Any]]) -> "GuidedSpec":
        return cls(tool_call_ast(tools))

    @classmethod
    def tool_call_tail(cls, tool: Dict[str, Any]) -> "tuple[str, GuidedSpec]":
        """One forced tool: the call's fixed head ``{"name": "<tool>", "parameters": ``
        (the agent writes it into the prompt as the start of the assistant turn, so
        it costs one prefill instead of a decode step per token) and the grammar of
        the rest of the call (``tool_call_ast`` minus that head)."""
        fn = tool.get("function", tool)
        head = '{"name": ' + json.dumps(fn["name"]) + ', "parameters": '
        rest = seq(schema_ast(fn.get("parameters") or {"type": "object"}, 1), lit("}"))
        more, tail = _peel_literal(rest)
        if tail is None:  # an all-literal call: keep a grammar to end it with
            return head, cls(rest)
        return head + more.decode("utf-8"), cls(tail)
