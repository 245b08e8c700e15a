"""CPU tests of the native C++ runtime (``_rt``): the prefix-caching KV block
manager, the UTF-8-safe incremental detokenizer and the JSON token FSM.
Property tests (hypothesis) check the allocator invariants the scheduler relies
on ("scheduler/KV allocator invariants")."""
import json

import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from fasttalk_llm_microservice_amd.engine import guided
from fasttalk_llm_microservice_amd.engine.tokenizer import get_tokenizer
from fasttalk_llm_microservice_amd.runtime import rt


# ----------------------------------------------------------------------------- blocks
def test_block_manager_basic_prefix_reuse():
    R = rt()
    bm = R.BlockManager(16, 4, True)
    toks = np.arange(13, dtype=np.int32)
    blocks = bm.allocate(4)
    assert len(blocks) == 4 and bm.num_free() == 12
    bm.commit(blocks, toks, 13, 0)  # 3 full blocks hashed
    assert bm.num_cached() == 3
    bm.free(blocks)
    assert bm.num_free() == 16  # cached blocks count as free (LRU)
    hit = bm.match_prefix(toks, 3)
    assert list(hit) == blocks[:3]
    assert all(bm.refcount(b) == 1 for b in hit)
    # different continuation of the first block only shares block 0
    other = toks.copy()
    other[5] = 999
    bm.free(hit)
    hit2 = bm.match_prefix(other, 3)
    assert list(hit2) == blocks[:1]
    bm.free(hit2)
    assert bm.hits == 4 and bm.queries == 5  # the lookup stops at the first miss


def test_block_manager_disabled_prefix_cache():
    bm = rt().BlockManager(8, 4, False)
    toks = np.arange(8, dtype=np.int32)
    b = bm.allocate(2)
    bm.commit(b, toks, 8, 0)
    bm.free(b)
    assert bm.match_prefix(toks, 2) == [] and bm.num_free() == 8


def test_block_manager_eviction_prefers_uncached():
    bm = rt().BlockManager(4, 2, True)
    b = bm.allocate(2)
    bm.commit(b, np.arange(4, dtype=np.int32), 4, 0)
    bm.free(b)
    fresh = bm.allocate(2)
    assert set(fresh).isdisjoint(b)  # never-hashed blocks go first
    assert bm.num_cached() == 2
    more = bm.allocate(2)  # now the LRU cached blocks are evicted
    assert set(more) == set(b) and bm.num_cached() == 0
    assert bm.allocate(1) == []


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(["alloc", "free", "match"]), st.integers(0, 40),
                          st.integers(0, 3)), max_size=60))
def test_block_manager_refcount_invariants(ops):
    """Random alloc/commit/free/match sequences: every block is either owned
    (refcount > 0) or free, free count + owned count == total, and a matched
    prefix always reproduces the committed tokens."""
    N, BS = 24, 4
    bm = rt().BlockManager(N, BS, True)
    owned = []  # (blocks, tokens)
    for op, n, which in ops:
        if op == "alloc":
            need = (n + BS - 1) // BS
            if not bm.can_allocate(need) or need == 0:
                continue
            blocks = bm.allocate(need)
            toks = (np.arange(n, dtype=np.int32) * (which + 1)) % 7
            bm.commit(blocks, toks, n, 0)
            owned.append((blocks, toks))
        elif op == "free" and owned:
            blocks, _ = owned.pop(which % len(owned))
            bm.free(blocks)
        elif op == "match":
            toks = (np.arange(n, dtype=np.int32) * (which + 1)) % 7
            hit = bm.match_prefix(toks, n // BS)
            assert len(hit) <= n // BS
            owned.append((list(hit), toks[: len(hit) * BS]))
        refs = {}
        for blocks, _ in owned:
            for b in blocks:
                refs[b] = refs.get(b, 0) + 1
        for b, r in refs.items():
            assert bm.refcount(b) == r
        assert bm.num_free() + len(refs) == N
    for blocks, _ in owned:
        bm.free(blocks)
    assert bm.num_free() == N


# ----------------------------------------------------------------------------- detok
def test_detokenizer_utf8_streaming():
    tok = get_tokenizer()
    d = rt().Detokenizer(tok.id_to_bytes)
    text = "Grüße aus Köln — 東京 🚀 done."
    ids = tok.encode(text)
    sid = d.new_stream()
    pieces = [d.push(sid, i) for i in ids] + [d.flush(sid)]
    assert "".join(pieces) == text
    for p in pieces:  # every emitted piece is valid UTF-8 text (no partial code points)
        p.encode("utf-8")
    assert d.decode(ids) == text
    d.release(sid)


def test_detokenizer_push_many_and_invalid_bytes():
    tok = get_tokenizer()
    d = rt().Detokenizer(tok.id_to_bytes)
    a, b = d.new_stream(), d.new_stream()
    ia, ib = tok.encode("hello"), tok.encode("world!")
    out_a, out_b = [], []
    for k in range(max(len(ia), len(ib))):
        sids, toks = [], []
        if k < len(ia):
            sids.append(a)
            toks.append(ia[k])
        if k < len(ib):
            sids.append(b)
            toks.append(ib[k])
        res = d.push_many(sids, toks)
        for s, r in zip(sids, res):
            (out_a if s == a else out_b).append(r)
    assert "".join(out_a) + d.flush(a) == "hello"
    assert "".join(out_b) + d.flush(b) == "world!"
    # a lone continuation byte becomes U+FFFD instead of breaking the stream
    bad = [i for i, bb in enumerate(tok.id_to_bytes) if bb == b"\x80"]
    if bad:
        s = d.new_stream()
        txt = d.push(s, bad[0]) + d.flush(s)
        assert txt == "�"


# ----------------------------------------------------------------------------- json fsm
def _walk_greedy(g, trie_tok, state, rng, max_steps=400):
    """Follow random allowed tokens until EOS is allowed and chosen."""
    out = []
    for _ in range(max_steps):
        mask = np.frombuffer(g.mask(state), dtype=np.uint32)
        allowed = np.nonzero(np.unpackbits(mask.view(np.uint8), bitorder="little"))[0]
        assert len(allowed) > 0
        t = int(rng.choice(allowed))
        if g.is_eos(t):
            assert g.accepting(state)
            return out
        out.append(t)
        state = g.advance_token(state, t)
        assert state >= 0
    raise AssertionError("grammar did not terminate")


@pytest.mark.parametrize("schema", [
    {"type": "object", "properties": {"city": {"type": "string", "maxLength": 12},
                                      "days": {"type": "integer"},
                                      "metric": {"type": "boolean"}}},
    {"type": "object", "properties": {"tags": {"type": "array", "items": {"type": "string",
                                                                          "maxLength": 5},
                                               "maxItems": 3},
                                      "mode": {"enum": ["fast", "slow"]},
                                      "score": {"type": "number"}},
     "required": ["tags", "mode", "score"]},
])
def test_json_grammar_random_walks_produce_valid_json(schema):
    tok = get_tokenizer()
    trie = rt().TokenTrie(tok.id_to_bytes)
    eos = [tok.eot_id, tok.eom_id]
    g = rt().Grammar(guided.schema_ast(schema), trie, eos)
    rng = np.random.default_rng(0)
    for _ in range(5):
        ids = _walk_greedy(g, trie, g.initial(), rng)
        obj = json.loads(tok.decode(ids))
        assert set(obj) == set(schema["properties"])
        if "mode" in obj:
            assert obj["mode"] in ("fast", "slow")
            assert isinstance(obj["tags"], list) and len(obj["tags"]) <= 3


def test_tool_call_grammar():
    tok = get_tokenizer()
    tools = [{"type": "function", "function": {"name": "get_current_time", "parameters": {
        "type": "object", "properties": {}}}},
        {"type": "function", "function": {"name": "duckduckgo_search", "parameters": {
            "type": "object", "properties": {"query": {"type": "string"}},
            "required": ["query"]}}}]
    g = rt().Grammar(guided.tool_call_ast(tools), rt().TokenTrie(tok.id_to_bytes),
                     [tok.eot_id, tok.eom_id])
    s = g.advance_bytes(g.initial(), b'{"name": "duckduckgo_search", "parameters": {"query": "x"}}')
    assert s >= 0 and g.accepting(s)
    assert g.advance_bytes(g.initial(), b'{"name": "nope"') == -1
    rng = np.random.default_rng(1)
    for _ in range(4):
        text = tok.decode(_walk_greedy(g, None, g.initial(), rng))
        obj = json.loads(text)
        assert obj["name"] in ("get_current_time", "duckduckgo_search")
        if obj["name"] == "duckduckgo_search":
            assert isinstance(obj["parameters"]["query"], str)
    assert g.num_allowed(g.initial()) > 0


def test_runtime_module_identity():
    """Under tests/unit/test_sanitizers.py the instrumented build is the one in use."""
    import os

    want = os.environ.get("FT_RT_MODULE")
    if want:
        assert rt().__name__ == want
