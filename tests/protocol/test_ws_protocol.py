"""/ws/llm protocol and HTTP routes (Appendix B) against
the real service stack on the CPU backend: FastAPI app -> session/conversation
managers -> NativeHandler -> AsyncEngine (engine thread) -> tiny random-init
Llama.  Driven with Starlette's TestClient (reference behaviour:
app/core/websocket_server_vllm.py:143-637)."""
import json
import os

import pytest
from starlette.testclient import TestClient

from app.utils.config import Config
from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import AsyncEngine, LLMEngine

SESSION_CFG = {"system_prompt": "You are terse.", "temperature": 0.0, "max_tokens": 6,
               "ignore_eos": True}


@pytest.fixture(scope="module")
def engine():
    eng = AsyncEngine(LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=512,
                                             max_model_len=2048, max_num_seqs=16))).start()
    yield eng
    eng.shutdown()


def _config(monkeypatch, **env):
    base = {"LLM_PROVIDER": "native", "ENABLE_PYDANTIC_AI": "false", "COMPUTE_DEVICE": "cpu",
            "LLM_MAX_CONNECTIONS": "4"}
    base.update(env)
    for k, v in base.items():
        monkeypatch.setenv(k, v)
    return Config()


@pytest.fixture()
def server(monkeypatch, engine):
    from app.core.websocket_server_vllm import WebSocketLLMServer

    return WebSocketLLMServer(_config(monkeypatch), engine=engine)


def _recv_until(ws, kind, limit=200):
    frames = []
    for _ in range(limit):
        f = ws.receive_json()
        frames.append(f)
        if f["type"] == kind:
            return frames
    raise AssertionError(f"no {kind} frame in {frames[-5:]}")


def test_http_routes(server):
    c = TestClient(server.app)
    r = c.get("/").json()
    assert r["service"] == "FastTalk LLM Service" and r["status"] == "ready" and r["provider"] == "native"
    h = c.get("/health")
    assert h.status_code == 200 and h.json()["status"] == "healthy" and h.json()["backend_connection"]
    st = c.get("/stats").json()
    assert set(st) >= {"connections", "conversations", "errors", "provider", "pydantic_ai_enabled"}
    assert set(st["errors"]["by_category"]) >= {"connection", "gpu", "timeout", "validation"}
    assert "kv_usage" in st["engine"]
    m = c.get("/models").json()
    assert m["current_model"] == "tiny" and m["models"] == ["tiny"]  # vLLM-path shape


def test_full_session_flow(server):
    c = TestClient(server.app)
    with c.websocket_connect("/ws/llm") as ws:
        hello = ws.receive_json()
        assert hello["type"] == "session_started" and hello["provider"] == "native"
        assert set(hello) == {"type", "session_id", "provider", "model", "pydantic_ai_enabled"}
        ws.send_json({"type": "start_session", "config": SESSION_CFG})
        conf = ws.receive_json()
        assert conf == {"type": "session_configured", "config": SESSION_CFG, "provider": "native"}
        ws.send_json({"type": "user_message", "text": "Hello there, how are you today?"})
        frames = _recv_until(ws, "response_complete")
        toks = [f for f in frames if f["type"] == "token"]
        assert toks and all(isinstance(f["data"], str) for f in toks)
        stats = frames[-1]["stats"]
        assert stats["tokens_generated"] == 6 and stats["provider"] == "native"
        assert {"processing_time_ms", "tokens_per_second", "pydantic_ai_used", "ttft_ms", "itl_ms"} <= set(stats)
        # second turn: the first turn's KV blocks are reused (multi-turn prefix cache)
        ws.send_json({"type": "user_message", "text": "And tomorrow?"})
        stats2 = _recv_until(ws, "response_complete")[-1]["stats"]
        assert stats2["cached_prompt_tokens"] > 0 and stats2["prompt_tokens"] > stats["prompt_tokens"]
        ws.send_json({"type": "end_session"})
        ended = ws.receive_json()
        assert ended["type"] == "session_ended"
        assert {"session_id", "messages_received", "tokens_generated", "config"} <= set(ended["stats"])
        assert ended["stats"]["tokens_generated"] == 12
    st = c.get("/stats").json()
    assert st["connections"]["total_generations_completed"] >= 2


def test_error_frames_and_idle_cancel(server):
    c = TestClient(server.app)
    with c.websocket_connect("/ws/llm") as ws:
        ws.receive_json()
        ws.send_text("{not json")
        assert ws.receive_json()["error"]["code"] == "invalid_json"
        ws.send_json({"type": "bogus"})
        assert ws.receive_json()["error"]["code"] == "unknown_message_type"
        ws.send_json({"type": "user_message", "text": ""})
        assert ws.receive_json()["error"]["code"] == "empty_message"
        ws.send_json({"type": "cancel"})
        assert ws.receive_json() == {"type": "cancelled", "success": False}
        ws.send_json({"type": "update_config", "config": {"temperature": 0.1, "max_tokens": 3}})
        upd = ws.receive_json()
        assert upd["type"] == "config_updated" and upd["success"] is True


def test_cancel_mid_stream_frees_kv(server, engine):
    c = TestClient(server.app)
    with c.websocket_connect("/ws/llm") as ws:
        ws.receive_json()
        ws.send_json({"type": "start_session", "config": dict(SESSION_CFG, max_tokens=400)})
        ws.receive_json()
        ws.send_json({"type": "user_message", "text": "Tell me a very long story."})
        first = ws.receive_json()
        assert first["type"] == "token"
        ws.send_json({"type": "cancel"})
        frames = _recv_until(ws, "cancelled")
        assert frames[-1]["success"] is True
        done = _recv_until(ws, "response_complete")[-1]
        assert done["stats"]["tokens_generated"] < 400 and done["stats"]["finish_reason"] == "abort"
    inner = engine.engine
    assert not inner.scheduler.running and not inner.scheduler.waiting


def test_max_connections(monkeypatch, engine):
    from app.core.websocket_server_vllm import WebSocketLLMServer

    srv = WebSocketLLMServer(_config(monkeypatch, LLM_MAX_CONNECTIONS="1"), engine=engine)
    c = TestClient(srv.app)
    with c.websocket_connect("/ws/llm") as ws1:
        ws1.receive_json()
        with c.websocket_connect("/ws/llm") as ws2:
            err = ws2.receive_json()
            assert err["type"] == "error" and err["error"]["code"] == "max_connections"
            assert err["error"]["severity"] == "high"


def test_v1_server_frame_shapes(monkeypatch, engine):
    from app.core.websocket_server import WebSocketLLMServer as V1

    srv = V1(_config(monkeypatch), engine=engine)
    c = TestClient(srv.app)
    assert c.get("/").json()["version"] == "1.0.0"
    with c.websocket_connect("/ws/llm") as ws:
        hello = ws.receive_json()
        assert set(hello) == {"type", "session_id"}
        ws.send_json({"type": "start_session", "config": SESSION_CFG})
        assert ws.receive_json() == {"type": "session_configured", "config": SESSION_CFG}
        ws.send_json({"type": "user_message", "text": "hi"})
        stats = _recv_until(ws, "response_complete")[-1]["stats"]
        assert set(stats) == {"tokens_generated", "processing_time_ms", "tokens_per_second"}
        ws.send_json({"type": "update_config", "config": {}})
        assert ws.receive_json()["error"]["code"] == "unknown_message_type"


def test_concurrent_sessions_batch_together(server, engine):
    """Several sessions in flight at once share engine steps (continuous batching)."""
    c = TestClient(server.app)
    inner = engine.engine
    before = inner.stats["decode_steps"]
    socks = [c.websocket_connect("/ws/llm") for _ in range(3)]
    wss = [s.__enter__() for s in socks]
    try:
        for ws in wss:
            ws.receive_json()
            ws.send_json({"type": "start_session", "config": dict(SESSION_CFG, max_tokens=12)})
            ws.receive_json()
        for i, ws in enumerate(wss):
            ws.send_json({"type": "user_message", "text": f"Question number {i}?"})
        for ws in wss:
            assert _recv_until(ws, "response_complete")[-1]["stats"]["tokens_generated"] == 12
    finally:
        for s in socks:
            s.__exit__(None, None, None)
    steps = inner.stats["decode_steps"] + inner.stats["mixed_steps"] - before
    assert steps < 3 * 12  # fewer engine steps than serial generation would need
