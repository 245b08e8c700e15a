"""CPU tests of the text front end: synthetic Llama-3 tokenizer, Llama-3.1 chat
template (prefix stability across turns -> KV reuse), tool-call parsers
(llama3_json + hermes, reference docker-compose.vllm.yml:50-51) and the
JSON-schema lowering used for guided tool calls."""
import json

import pytest

from fasttalk_llm_microservice_amd.engine import guided
from fasttalk_llm_microservice_amd.engine.chat_template import ChatTemplate, render_tools
from fasttalk_llm_microservice_amd.engine.tokenizer import get_tokenizer
from fasttalk_llm_microservice_amd.engine.tool_parser import (StreamingToolDetector, ToolCall,
                                                              parse_hermes, parse_llama3_json,
                                                              parse_tool_calls)


@pytest.fixture(scope="module")
def tok():
    return get_tokenizer()


def test_tokenizer_llama3_specials(tok):
    assert tok.vocab_size == 128256
    assert (tok.bos_id, tok.eos_id, tok.eot_id, tok.eom_id) == (128000, 128001, 128009, 128008)
    assert (tok.start_header_id, tok.end_header_id, tok.python_tag_id) == (128006, 128007, 128010)
    assert tok.stop_ids == [128001, 128008, 128009]
    assert tok.is_special(128009) and not tok.is_special(1000)


@pytest.mark.parametrize("text", ["Hello, world!", "  leading spaces\nand\ttabs",
                                  "naïve café — 東京 🚀", "{\"json\": [1, 2.5, null]}", ""])
def test_tokenizer_roundtrip(tok, text):
    ids = tok.encode(text)
    assert all(0 <= i < 128000 for i in ids)
    assert tok.decode(ids) == text
    assert b"".join(tok.id_to_bytes[i] for i in ids).decode("utf-8") == text


def test_chat_template_format_and_prefix_stability(tok):
    ct = ChatTemplate(tok)
    conv = [{"role": "system", "content": "Be brief."}, {"role": "user", "content": "Hi"}]
    ids = ct.render(conv)
    assert ids[0] == tok.bos_id
    text = ct.render_text(conv)
    assert text == ("<|begin_of_text|><|start_header_id|>system<|end_header_id|>\n\nBe brief."
                    "<|eot_id|><|start_header_id|>user<|end_header_id|>\n\nHi<|eot_id|>"
                    "<|start_header_id|>assistant<|end_header_id|>\n\n")
    # the next turn's prompt starts with this turn's prompt + reply: prefix-cache friendly
    conv2 = conv + [{"role": "assistant", "content": "Hello!"}, {"role": "user", "content": "More"}]
    ids2 = ct.render(conv2)
    assert ids2[: len(ids)] == ids
    no_gen = ct.render(conv, add_generation_prompt=False)
    assert ids[: len(no_gen)] == no_gen and len(ids) > len(no_gen)


def test_chat_template_tools_and_tool_messages(tok):
    ct = ChatTemplate(tok)
    tools = [{"type": "function", "function": {"name": "get_current_time", "description": "t",
                                               "parameters": {"type": "object", "properties": {}}}}]
    msgs = [{"role": "system", "content": "S"}, {"role": "user", "content": "time?"},
            {"role": "assistant", "content": None, "tool_calls": [
                {"id": "c1", "type": "function",
                 "function": {"name": "get_current_time", "arguments": "{}"}}]},
            {"role": "tool", "tool_call_id": "c1", "content": "noon"}]
    text = ct.render_text(msgs, tools=tools)
    assert render_tools(tools) in text and text.index(render_tools(tools)) < text.index("S<|eot_id|>")
    assert '{"name": "get_current_time", "parameters": {}}' in text
    assert "<|start_header_id|>ipython<|end_header_id|>\n\nnoon<|eot_id|>" in text


def test_parse_llama3_json_variants():
    calls = parse_llama3_json('<|python_tag|>{"name": "a", "parameters": {"x": 1}}; '
                              '{"name": "b", "arguments": "{\\"y\\": 2}"}')
    assert [(c.name, c.arguments) for c in calls] == [("a", {"x": 1}), ("b", {"y": 2})]
    assert parse_llama3_json("just words") == []
    assert parse_llama3_json('{"name": "a", "parameters": {') == []
    assert parse_llama3_json('{"no_name": 1}') == []


def test_parse_hermes_and_auto():
    text = 'Sure. <tool_call>{"name": "s", "arguments": {"query": "q"}}</tool_call> done'
    calls = parse_hermes(text)
    assert calls[0].name == "s" and calls[0].arguments == {"query": "q"}
    calls, rest = parse_tool_calls(text)
    assert len(calls) == 1 and rest == "Sure.  done"
    calls, rest = parse_tool_calls('{"name": "t", "parameters": {}}')
    assert calls[0].name == "t" and rest == ""
    calls, rest = parse_tool_calls("hello", fmt="hermes")
    assert calls == [] and rest == "hello"
    oa = ToolCall("n", {"a": 1}).to_openai()
    assert oa["type"] == "function" and json.loads(oa["function"]["arguments"]) == {"a": 1}


def test_streaming_tool_detector():
    d = StreamingToolDetector()
    assert d.feed("  ") == (None, "")
    assert d.feed("Hel") == ("text", "  Hel")
    assert d.feed("lo") == ("text", "lo")
    d = StreamingToolDetector()
    assert d.feed("<|pyth") == (None, "")
    assert d.feed("on_tag|>{") == ("tool", "")
    d = StreamingToolDetector()
    assert d.feed('{"name"') == ("tool", "") and d.buf == '{"name"'


def test_schema_ast_shapes():
    ast = guided.schema_ast({"type": "object", "properties": {"a": {"type": "integer"}}})
    assert ast["t"] == "seq" and ast["c"][0] == guided.lit("{")
    assert guided.schema_ast({"enum": ["x", 1]}) == guided.alt(guided.lit('"x"'), guided.lit("1"))
    assert guided.schema_ast({}) == guided.lit("{}")
    spec = guided.GuidedSpec.json_schema({"type": "boolean"})
    assert spec.key == guided.GuidedSpec.json_schema({"type": "boolean"}).key
