"""BASELINE config 1: "llama3.2:1b single-session greedy stream over /ws/llm on
CPU backend (plumbing, no GPU)".  The service is built the way `main.py` builds it
-- the Ollama-style model tag from the reference's configuration
(`/root/reference/app/utils/config.py:86`, LLM_MODEL=llama3.2:1b) resolved by
the native provider to the Llama-3.2-1B architecture (16 layers, hidden 2048,
GQA 32/8, tied embeddings) with random-init weights on the CPU -- and one
session streams a greedy reply over the real WebSocket protocol."""
import pytest
from starlette.testclient import TestClient

from app.utils.config import Config


@pytest.fixture(scope="module")
def server():
    mp = pytest.MonkeyPatch()
    for k, v in {"LLM_PROVIDER": "native", "LLM_MODEL": "llama3.2:1b", "ENABLE_PYDANTIC_AI": "false",
                 "COMPUTE_DEVICE": "cpu", "ENGINE_MAX_MODEL_LEN": "512", "ENGINE_NUM_KV_BLOCKS": "64",
                 "ENGINE_MAX_NUM_SEQS": "2", "LLM_MAX_CONNECTIONS": "2"}.items():
        mp.setenv(k, v)
    mp.delenv("ENGINE_MODEL", raising=False)
    from app.core.websocket_server_vllm import WebSocketLLMServer

    srv = WebSocketLLMServer(Config())
    yield srv
    try:
        srv.native_handler.engine.shutdown()
    finally:
        mp.undo()


def _stream(ws, text):
    ws.send_json({"type": "user_message", "text": text})
    frames = []
    for _ in range(200):
        f = ws.receive_json()
        frames.append(f)
        if f["type"] in ("response_complete", "error"):
            return frames
    raise AssertionError(frames[-3:])


def test_llama32_1b_greedy_stream_over_ws_on_cpu(server):
    eng = server.native_handler.engine
    info = eng.model_info()
    assert info["model"] == "llama3.2-1b" and info["num_layers"] == 16
    assert info["hidden_size"] == 2048 and info["num_kv_heads"] == 8
    cfg = {"system_prompt": "You are terse.", "temperature": 0.0, "max_tokens": 6, "ignore_eos": True}
    c = TestClient(server.app)
    with c.websocket_connect("/ws/llm") as ws:
        assert ws.receive_json()["type"] == "session_started"
        ws.send_json({"type": "start_session", "config": cfg})
        assert ws.receive_json()["type"] == "session_configured"
        a = _stream(ws, "Say something short.")
        assert a[-1]["type"] == "response_complete", a[-1]
        st = a[-1]["stats"]
        assert st["tokens_generated"] == 6 and st["provider"] == "native"
        toks = "".join(f["data"] for f in a if f["type"] == "token")
        # second turn reuses the first turn's KV through the prefix cache
        b = _stream(ws, "And again.")
        assert b[-1]["type"] == "response_complete"
        assert b[-1]["stats"]["cached_prompt_tokens"] > 0
    # greedy: the same first turn in a fresh session streams the same text
    with c.websocket_connect("/ws/llm") as ws:
        ws.receive_json()
        ws.send_json({"type": "start_session", "config": cfg})
        ws.receive_json()
        a2 = _stream(ws, "Say something short.")
        assert "".join(f["data"] for f in a2 if f["type"] == "token") == toks
