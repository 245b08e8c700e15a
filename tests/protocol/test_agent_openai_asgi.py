"""Agent loop (BASELINE config 5: tool calling + web-search stub with guided JSON
tool calls on random weights), the OpenAI-compatible facade, the aiohttp ASGI
transport (real sockets on 127.0.0.1) and the monitoring service, all on the
CPU backend.  Reference behaviour: app/agents/voice_agent.py:147-344,
app/monitoring/service_monitor.py:85-137."""
import asyncio
import json
from datetime import datetime

import pytest
from starlette.testclient import TestClient

from app.agents.tools import make_search_tool, make_session_tool, make_time_tool
from app.agents.voice_agent import AgentConfig, ConversationContext, VoiceAgent
from app.core.native_handler import NativeHandler
from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import AsyncEngine, LLMEngine


@pytest.fixture(scope="module")
def engine():
    eng = AsyncEngine(LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=512,
                                             max_model_len=2048, max_num_seqs=16))).start()
    yield eng
    eng.shutdown()


def _ctx(sid="s1"):
    return ConversationContext(user_id="u", session_id=sid, conversation_history=[],
                               created_at=datetime.now())


# ----------------------------------------------------------------------------- tools
def test_tools_offline():
    search = make_search_tool(rate_limit=0.0, backend="stub")
    res = json.loads(asyncio.run(search(None, query="mi355x hbm", max_results=3)))
    assert len(res) == 3 and {"title", "href", "body"} <= set(res[0])
    assert "current date" in asyncio.run(make_time_tool()(None))
    info = asyncio.run(make_session_tool()(_ctx("abcdefghij")))
    assert info.startswith("Session abcdefgh...")
    assert search.schema()["function"]["parameters"]["required"] == ["query"]


# ----------------------------------------------------------------------------- agent
def test_agent_guided_tool_call_round_trip(engine):
    handler = NativeHandler(engine=engine)
    agent = VoiceAgent(AgentConfig(guided_tool_calls=True, max_tokens=24, temperature=0.7,
                                   tool_round_priority=1), backend=handler)
    assert agent.is_native and set(agent.tools()) == {"duckduckgo_search", "get_current_time",
                                                       "get_session_info"}

    prios = []
    orig = engine.generate

    def spy(prompt_ids, params, request_id=None):
        prios.append((params.guided is not None, params.priority))
        return orig(prompt_ids, params, request_id=request_id)

    async def run():
        return [ev async for ev in agent.generate_events("Search the web for the weather news",
                                                         _ctx(), seed=5, max_tokens=24)]

    engine.generate = spy
    try:
        events = asyncio.run(run())
    finally:
        engine.generate = orig
    calls = [e for e in events if e.tool_call]
    assert calls, "guided decoding must produce a valid tool call"
    assert calls[0].tool_call["name"] in agent.tools() and calls[0].tool_result
    assert events[-1].finish_reason in ("stop", "length")
    # the forced call keeps arrival order; the re-prompt after the tool jumps the queue
    # (AGENT_TOOL_ROUND_PRIORITY, opt-in)
    assert prios[0] == (True, 0) and len(prios) >= 2 and prios[1][1] == 1, prios


@pytest.mark.parametrize("head", [True, False])
def test_agent_plain_answer_and_custom_tool(engine, head):
    """tool_choice names one tool: with prefill_tool_head its call's fixed head is
    written into the prompt and only the arguments are decoded under the grammar."""
    handler = NativeHandler(engine=engine)
    agent = VoiceAgent(AgentConfig(guided_tool_calls=False, prefill_tool_head=head), backend=handler)
    prompts = []
    orig = engine.generate

    def spy(prompt_ids, params, request_id=None):
        prompts.append((list(prompt_ids), params.guided is not None))
        return orig(prompt_ids, params, request_id=request_id)

    engine.generate = spy

    @agent.tool(description="Adds two numbers", parameters={
        "type": "object", "properties": {"a": {"type": "integer"}, "b": {"type": "integer"}}})
    def add(ctx, a, b):
        return str(a + b)

    assert "add" in agent.tools()

    async def run():
        evs = [ev async for ev in agent.generate_events("add please", _ctx("s2"), temperature=0.0,
                                                        max_tokens=8, tool_choice="add", seed=1)]
        return evs

    try:
        evs = asyncio.run(run())
    finally:
        engine.generate = orig
    call = [e for e in evs if e.tool_call][0]
    assert call.tool_call["name"] == "add"
    guided_prompt = [p for p, g in prompts if g][0]
    from fasttalk_llm_microservice_amd.engine.guided import GuidedSpec

    head_text = GuidedSpec.tool_call_tail(agent.tools()["add"].schema())[0]
    assert head_text == '{"name": "add", "parameters": {"a": '
    tail = handler.tokenizer.encode(head_text)
    assert (guided_prompt[-len(tail):] == tail) == head
    a, b = call.tool_call["arguments"]["a"], call.tool_call["arguments"]["b"]
    assert call.tool_result == str(a + b)
    info = agent.get_model_info()
    assert info["base_url"] == "in-process" and "add" in info["tools"]


def test_ws_agent_path(monkeypatch, engine):
    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.utils.config import Config

    for k, v in {"LLM_PROVIDER": "native", "ENABLE_PYDANTIC_AI": "true",
                 "COMPUTE_DEVICE": "cpu"}.items():
        monkeypatch.setenv(k, v)
    srv = WebSocketLLMServer(Config(), engine=engine)
    c = TestClient(srv.app)
    assert c.get("/").json()["pydantic_ai_enabled"] is True
    with c.websocket_connect("/ws/llm") as ws:
        assert ws.receive_json()["pydantic_ai_enabled"] is True
        ws.send_json({"type": "start_session", "config": {"max_tokens": 5, "temperature": 0.0,
                                                          "ignore_eos": True}})
        ws.receive_json()
        ws.send_json({"type": "user_message", "text": "hello"})
        while True:
            f = ws.receive_json()
            if f["type"] == "response_complete":
                break
        assert f["stats"]["pydantic_ai_used"] is True and f["stats"]["tokens_generated"] >= 1
        ws.send_json({"type": "update_config", "config": {"enable_web_search": False}})
        assert ws.receive_json()["type"] == "config_updated"
    assert "duckduckgo_search" not in srv.voice_agent.tools()


# ----------------------------------------------------------------------------- openai facade
def test_openai_chat_completions(monkeypatch, engine):
    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.utils.config import Config

    monkeypatch.setenv("LLM_PROVIDER", "native")
    monkeypatch.setenv("ENABLE_PYDANTIC_AI", "false")
    c = TestClient(WebSocketLLMServer(Config(), engine=engine).app)
    assert c.get("/v1/models").json()["data"][0]["id"] == "tiny"
    body = {"messages": [{"role": "user", "content": "hi"}], "max_tokens": 5, "temperature": 0,
            "ignore_eos": True}
    r = c.post("/v1/chat/completions", json=body).json()
    assert r["object"] == "chat.completion" and r["usage"]["completion_tokens"] == 5
    assert r["choices"][0]["finish_reason"] == "length"
    s = c.post("/v1/chat/completions", json=dict(body, stream=True))
    lines = [x for x in s.text.split("\n\n") if x]
    assert lines[-1] == "data: [DONE]" and json.loads(lines[0][6:])["object"] == "chat.completion.chunk"
    tools = [{"type": "function", "function": {"name": "get_weather", "parameters": {
        "type": "object", "properties": {"city": {"type": "string", "maxLength": 10}}}}}]
    r = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "w?"}],
                                             "tools": tools, "tool_choice": "required",
                                             "max_tokens": 40, "seed": 3}).json()
    msg = r["choices"][0]["message"]
    assert r["choices"][0]["finish_reason"] == "tool_calls"
    assert msg["tool_calls"][0]["function"]["name"] == "get_weather"
    assert "city" in json.loads(msg["tool_calls"][0]["function"]["arguments"])
    rf = {"type": "json_schema", "json_schema": {"schema": {
        "type": "object", "properties": {"ok": {"type": "boolean"}}}}}
    r = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "j"}],
                                             "response_format": rf, "max_tokens": 20}).json()
    assert isinstance(json.loads(r["choices"][0]["message"]["content"])["ok"], bool)
    assert c.post("/v1/chat/completions", json={"messages": []}).status_code == 400


def _sse(text):
    out = []
    for x in text.split("\n\n"):
        if x.startswith("data: ") and x != "data: [DONE]":
            out.append(json.loads(x[6:]))
    return out


def test_openai_streams_with_tools(monkeypatch, engine):
    """with ``tools`` the facade streams -- speech as content deltas
    before finish_reason, tool calls as incremental delta.tool_calls (id + name
    first, then argument fragments), like vLLM's auto tool choice that the
    reference consumes (/root/reference/app/core/vllm_handler.py:389-408)."""
    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.utils.config import Config

    monkeypatch.setenv("LLM_PROVIDER", "native")
    monkeypatch.setenv("ENABLE_PYDANTIC_AI", "false")
    c = TestClient(WebSocketLLMServer(Config(), engine=engine).app)
    tools = [{"type": "function", "function": {"name": "get_weather", "parameters": {
        "type": "object", "properties": {"city": {"type": "string", "maxLength": 12}}}}}]
    # tool call: forced by tool_choice, streamed incrementally
    s = c.post("/v1/chat/completions", json={
        "messages": [{"role": "user", "content": "weather?"}], "tools": tools,
        "tool_choice": "required", "max_tokens": 48, "seed": 3, "stream": True})
    chunks = _sse(s.text)
    tc = [ch["choices"][0]["delta"]["tool_calls"] for ch in chunks
          if "tool_calls" in ch["choices"][0]["delta"]]
    assert len(tc) >= 2, "tool call must stream in more than one chunk"
    first = tc[0][0]
    assert first["index"] == 0 and first["id"].startswith("call_")
    assert first["function"]["name"] == "get_weather" and first["function"]["arguments"] == ""
    args = "".join(d["function"]["arguments"] for deltas in tc for d in deltas if d["index"] == 0)
    assert "city" in json.loads(args)
    assert chunks[-1]["choices"][0]["finish_reason"] == "tool_calls"
    # speech: content chunks arrive one by one, before the finishing chunk
    s = c.post("/v1/chat/completions", json={
        "messages": [{"role": "user", "content": "say hi"}], "tools": tools,
        "max_tokens": 12, "temperature": 0, "ignore_eos": True, "stream": True})
    chunks = _sse(s.text)
    deltas = [ch["choices"][0]["delta"] for ch in chunks]
    fin = [i for i, ch in enumerate(chunks) if ch["choices"][0]["finish_reason"]]
    assert fin == [len(chunks) - 1]
    content = [i for i, d in enumerate(deltas) if d.get("content")]
    calls = [i for i, d in enumerate(deltas) if d.get("tool_calls")]
    # random weights decide whether the first characters look like a tool call;
    # either way the reply streams in several chunks before finish_reason
    assert len(content) >= 2 or len(calls) >= 1
    assert all(i < fin[0] for i in content + calls)


def test_openai_stream_json_text_with_tools_is_content(monkeypatch, engine):
    """with ``tools`` present, a reply that starts with '{' but is not a
    call of one of the request's tools (a JSON answer) is streamed as content."""
    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.utils.config import Config
    from fasttalk_llm_microservice_amd.engine.tool_parser import StreamingToolCallParser

    monkeypatch.setenv("LLM_PROVIDER", "native")
    monkeypatch.setenv("ENABLE_PYDANTIC_AI", "false")
    c = TestClient(WebSocketLLMServer(Config(), engine=engine).app)
    tools = [{"type": "function", "function": {"name": "get_weather", "parameters": {
        "type": "object", "properties": {"city": {"type": "string"}}}}}]
    rf = {"type": "json_schema", "json_schema": {"schema": {
        "type": "object", "properties": {"ok": {"type": "boolean"}}, "required": ["ok"]}}}
    s = c.post("/v1/chat/completions", json={
        "messages": [{"role": "user", "content": "json please"}], "tools": tools,
        "response_format": rf, "max_tokens": 20, "seed": 2, "stream": True})
    chunks = _sse(s.text)
    deltas = [ch["choices"][0]["delta"] for ch in chunks]
    assert not any(d.get("tool_calls") for d in deltas)
    text = "".join(d.get("content") or "" for d in deltas)
    assert isinstance(json.loads(text)["ok"], bool)
    assert chunks[-1]["choices"][0]["finish_reason"] in ("stop", "length")
    # a "name" that is not a requested tool never becomes a call header
    p = StreamingToolCallParser(["get_weather"])
    assert p.feed('{"name": "Alice", "parameters": {"a": 1}}') == [] and p.rejected
    p = StreamingToolCallParser(["get_weather"])
    out = p.feed('{"name": "get_weather", "parameters": {"city": "Oslo"}}')
    assert out[0]["function"]["name"] == "get_weather"


# ----------------------------------------------------------------------------- ASGI over aiohttp
def test_aiohttp_asgi_transport_serves_ws_and_http(monkeypatch, engine):
    import aiohttp

    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.server.asgi_aiohttp import AiohttpASGIServer
    from app.utils.config import Config

    monkeypatch.setenv("LLM_PROVIDER", "native")
    monkeypatch.setenv("ENABLE_PYDANTIC_AI", "false")
    srv = WebSocketLLMServer(Config(), engine=engine)

    async def main():
        asgi = AiohttpASGIServer(srv.app, "127.0.0.1", 0)
        await asgi.start()
        try:
            base = f"127.0.0.1:{asgi.port}"
            async with aiohttp.ClientSession() as s:
                async with s.get(f"http://{base}/health") as r:
                    assert r.status == 200 and (await r.json())["status"] == "healthy"
                async with s.ws_connect(f"ws://{base}/ws/llm") as ws:
                    hello = json.loads((await ws.receive()).data)
                    assert hello["type"] == "session_started"
                    await ws.send_str(json.dumps({"type": "start_session", "config": {
                        "max_tokens": 4, "temperature": 0, "ignore_eos": True}}))
                    await ws.receive()
                    await ws.send_str(json.dumps({"type": "user_message", "text": "yo"}))
                    n = 0
                    while True:
                        f = json.loads((await ws.receive()).data)
                        n += f["type"] == "token"
                        if f["type"] == "response_complete":
                            break
                    assert f["stats"]["tokens_generated"] == 4 and n >= 1
        finally:
            await asgi.stop()

    asyncio.run(main())


def test_v1_frames_hold_on_the_aiohttp_transport(monkeypatch, engine):
    """the v1 server's frame shapes (reference
    websocket_server.py:160-163) must survive the raw-socket send path of the
    production transport, not only Starlette's TestClient."""
    import aiohttp

    from app.core.websocket_server import WebSocketLLMServer as V1
    from app.server.asgi_aiohttp import AiohttpASGIServer
    from app.utils.config import Config

    monkeypatch.setenv("LLM_PROVIDER", "native")
    monkeypatch.setenv("ENABLE_PYDANTIC_AI", "false")
    srv = V1(Config(), engine=engine)

    async def main():
        asgi = AiohttpASGIServer(srv.app, "127.0.0.1", 0)
        await asgi.start()
        try:
            async with aiohttp.ClientSession() as s:
                async with s.get(f"http://127.0.0.1:{asgi.port}/health") as r:
                    h = await r.json()
                    assert "ollama_connection" in h and "provider" not in h
                async with s.ws_connect(f"ws://127.0.0.1:{asgi.port}/ws/llm") as ws:
                    hello = json.loads((await ws.receive()).data)
                    await ws.send_str(json.dumps({"type": "start_session", "config": {
                        "max_tokens": 3, "temperature": 0, "ignore_eos": True}}))
                    conf = json.loads((await ws.receive()).data)
                    await ws.send_str(json.dumps({"type": "user_message", "text": "hi"}))
                    while True:
                        f = json.loads((await ws.receive()).data)
                        if f["type"] == "response_complete":
                            break
                    await ws.send_str(json.dumps({"type": "update_config", "config": {}}))
                    err = json.loads((await ws.receive()).data)
                    return hello, conf, f, err
        finally:
            await asgi.stop()

    hello, conf, done, err = asyncio.run(main())
    assert set(hello) == {"type", "session_id"}
    assert set(conf) == {"type", "config"}
    assert set(done["stats"]) == {"tokens_generated", "processing_time_ms", "tokens_per_second"}
    assert done["stats"]["tokens_generated"] == 3
    assert err["type"] == "error" and err["error"]["code"] == "unknown_message_type"


# ----------------------------------------------------------------------------- monitoring
def test_service_monitor_metrics_and_prometheus(monkeypatch, engine):
    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.monitoring.service_monitor import MonitoringServer, ServiceMonitor, prometheus_text
    from app.utils.config import Config

    monkeypatch.setenv("LLM_PROVIDER", "native")
    monkeypatch.setenv("ENABLE_PYDANTIC_AI", "false")
    mon = ServiceMonitor()
    srv = WebSocketLLMServer(Config(), monitor=mon, engine=engine)
    mon.attach_server(srv)
    mon.record_request()
    mon.record_generation(10, 0.5, ttft=0.05)
    mon.record_error()
    m = mon.get_metrics()
    assert m["requests"] == 1 and m["generations"] == 1 and m["errors"] == 1
    assert m["total_tokens_generated"] == 10 and m["avg_processing_time_seconds"] == pytest.approx(0.5)
    txt = prometheus_text(m)
    assert "fasttalk_requests" in txt and "fasttalk_total_tokens_generated 10" in txt
    ms = MonitoringServer(port=19092, monitor=mon)
    c = ms.app.test_client()
    h = c.get("/health").get_json()
    assert h["status"] == "healthy" and "system" in h
    assert c.get("/health/ready").get_json() == {"status": "ready"}
    assert c.get("/health/live").get_json() == {"status": "live"}
    assert c.get("/metrics").get_json()["requests"] == 1
    assert c.get("/info").get_json()["service"] == "llm-service"
    assert b"fasttalk_requests" in c.get("/metrics/prometheus").data


def test_manual_client_scripted(monkeypatch, engine, capsys):
    """The shipped test_llm_client.py drives a real socket session end to end."""
    import test_llm_client

    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.server.asgi_aiohttp import AiohttpASGIServer
    from app.utils.config import Config

    monkeypatch.setenv("LLM_PROVIDER", "native")
    monkeypatch.setenv("ENABLE_PYDANTIC_AI", "false")
    srv = WebSocketLLMServer(Config(), engine=engine)

    async def main():
        asgi = AiohttpASGIServer(srv.app, "127.0.0.1", 0)
        await asgi.start()
        try:
            return await test_llm_client.run(f"ws://127.0.0.1:{asgi.port}/ws/llm", ["hello", "again"],
                                             {"max_tokens": 4, "temperature": 0.0, "ignore_eos": True})
        finally:
            await asgi.stop()

    assert asyncio.run(main()) == 0
    out = capsys.readouterr().out
    assert out.count("[4 tokens") == 2 and "session ended" in out


def test_tool_hints_force_one_tool_when_unambiguous(engine):
    agent = VoiceAgent(AgentConfig(guided_tool_calls=True), backend=NativeHandler(engine=engine))
    assert agent._wants_tool("Search the web for the latest news about tea", None) == "duckduckgo_search"
    assert agent._wants_tool("what time is it", None) == "get_current_time"
    assert agent._wants_tool("search for the date of the match", None) == "required"
    assert agent._wants_tool("what is the current weather", None) == "required"
    assert agent._wants_tool("tell me a story", None) is None
    assert agent._wants_tool("search news", "get_session_info") == "get_session_info"


# ----------------------------------------------------------------------------- remote provider
def _serve_facade(engine):
    """This repo's own OpenAI facade (/v1) on a real socket, in a thread."""
    import threading

    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.server.asgi_aiohttp import AiohttpASGIServer
    from app.utils.config import Config

    cfg = Config()
    cfg.llm_provider = "native"
    cfg.enable_pydantic_ai = False
    srv = WebSocketLLMServer(cfg, engine=engine)
    asgi = AiohttpASGIServer(srv.app, "127.0.0.1", 0)
    loop = asyncio.new_event_loop()
    ready = threading.Event()

    def run():
        asyncio.set_event_loop(loop)
        loop.run_until_complete(asgi.start())
        ready.set()
        loop.run_forever()

    threading.Thread(target=run, daemon=True).start()
    assert ready.wait(30)

    def stop():
        asyncio.run_coroutine_threadsafe(asgi.stop(), loop).result(15)
        loop.call_soon_threadsafe(loop.stop)
    return asgi.port, stop


def test_agent_tool_loop_over_remote_openai_provider(monkeypatch, engine):
    """LLM_PROVIDER=openai with VLLM_BASE_URL at this repo's own
    OpenAI facade (AiohttpASGIServer): the agent sends its tools with
    tool_choice="required", assembles the streamed tool_calls deltas, runs the tool,
    re-prompts with the result and streams the answer (reference
    app/agents/voice_agent.py:141-164,219-229 over vllm_handler.py)."""
    from app.core.vllm_handler import VLLMHandler

    monkeypatch.setenv("WEB_SEARCH_BACKEND", "stub")
    port, stop = _serve_facade(engine)
    try:
        base = f"http://127.0.0.1:{port}/v1"
        handler = VLLMHandler(base, "fasttalk-native")
        assert handler.check_connection()
        agent = VoiceAgent(AgentConfig(vllm_base_url=base, max_tokens=12, temperature=0.7,
                                       duckduckgo_rate_limit=0.0), backend=handler)
        assert not agent.is_native

        async def run(choice):
            return [ev async for ev in agent.generate_events(
                "Search the web for the latest tea news", _ctx("remote1"), tool_choice=choice,
                seed=3, max_tokens=12, ignore_eos=True)]

        events = asyncio.run(run("required"))
        calls = [e for e in events if e.tool_call]
        assert calls and calls[0].tool_call["name"] in agent.tools() and calls[0].tool_result
        after = events[events.index(calls[-1]) + 1:]
        assert sum(e.num_tokens for e in after if e.text) >= 1, "the answer must stream after the tool"
        assert events[-1].finish_reason in ("stop", "length")
        # a named tool: the server is told which one
        events = asyncio.run(run("get_current_time"))
        named = [e for e in events if e.tool_call]
        assert named and named[0].tool_call["name"] == "get_current_time"
        assert "current date" in named[0].tool_result
    finally:
        stop()


def test_ws_agent_over_remote_openai_provider(monkeypatch, engine):
    """The whole reference default path: /ws/llm -> VoiceAgent -> remote OpenAI API
    (this repo's facade) with guided tool calls for a search-worded message."""
    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.utils.config import Config

    monkeypatch.setenv("WEB_SEARCH_BACKEND", "stub")
    port, stop = _serve_facade(engine)
    try:
        for k, v in {"LLM_PROVIDER": "openai", "VLLM_BASE_URL": f"http://127.0.0.1:{port}/v1",
                     "ENABLE_PYDANTIC_AI": "true", "AGENT_GUIDED_TOOL_CALLS": "true",
                     "DUCKDUCKGO_RATE_LIMIT": "0"}.items():
            monkeypatch.setenv(k, v)
        srv = WebSocketLLMServer(Config())
        assert srv.voice_agent is not None and srv.vllm_handler is not None
        with TestClient(srv.app) as c, c.websocket_connect("/ws/llm") as ws:
            assert ws.receive_json()["type"] == "session_started"
            ws.send_json({"type": "start_session", "config": {"max_tokens": 10, "temperature": 0.7,
                                                              "seed": 1, "ignore_eos": True}})
            ws.receive_json()
            ws.send_json({"type": "user_message", "text": "Search the web for the weather news"})
            n = 0
            while True:
                f = ws.receive_json()
                if f["type"] == "token":
                    n += 1
                    continue
                assert f["type"] == "response_complete", f
                break
        assert n >= 1 and f["stats"]["tokens_generated"] >= 1 and f["stats"]["pydantic_ai_used"]
    finally:
        stop()
