"""Unit tests (CPU) for the service utilities that keep the reference's public API:
Config (reference app/utils/config.py), StructuredLogger (app/utils/logger.py),
ErrorHandler / CircuitBreaker / RetryManager (app/utils/error_handler.py),
ConnectionManager (app/utils/connection_manager.py), ConversationManager and
TextContext (app/core/conversation_manager.py, app/core/text_processor.py)."""
import asyncio
import json
import logging
import time

import pytest

from app.core.conversation_manager import ConversationManager, ConversationState
from app.core.text_processor import TextContext, calculate_text_similarity
from app.utils import config as cfgmod
from app.utils.config import Config, VALID_PROVIDERS
from app.utils.connection_manager import ConnectionManager, ConnectionState
from app.utils.error_handler import (CircuitBreaker, CircuitBreakerState, ErrorCategory,
                                     ErrorHandler, ErrorSeverity, LLMServiceError, RetryManager)
from app.utils.logger import JsonFormatter, StructuredLogger, request_context


# ----------------------------------------------------------------------------- config
def test_config_defaults_and_native_provider(monkeypatch):
    for k in ("LLM_PROVIDER", "LLM_PORT", "DEFAULT_TOP_P", "ENGINE_MODEL"):
        monkeypatch.delenv(k, raising=False)
    c = Config()
    assert c.llm_provider == "native" and "native" in VALID_PROVIDERS
    assert c.port == 8000 and c.monitoring_port == 9092 and c.max_connections == 50
    assert c.default_temperature == 0.7 and c.default_top_k == 40
    assert c.agent_json_tool_calls is False
    d = c.to_dict()
    assert d["llm_provider"] == "native" and "engine_model" in d and "engine_tp_size" in d


def test_config_env_overrides(monkeypatch):
    monkeypatch.setenv("LLM_PROVIDER", "vllm")
    monkeypatch.setenv("VLLM_MODEL", "my/model")
    monkeypatch.setenv("LLM_PORT", "9100")
    monkeypatch.setenv("DEFAULT_MAX_TOKENS", "64")
    monkeypatch.setenv("VLLM_TENSOR_PARALLEL_SIZE", "4")
    c = Config()
    assert c.llm_provider == "vllm" and c.current_model() == "my/model"
    assert c.port == 9100 and c.default_max_tokens == 64 and c.engine_tp_size == 4
    assert "vllm_base_url" in c.to_dict()


@pytest.mark.parametrize("var,val", [("DEFAULT_TOP_P", "1.5"), ("DEFAULT_TOP_K", "0"),
                                     ("DEFAULT_MAX_TOKENS", "0"), ("LLM_PORT", "80"),
                                     ("LLM_MONITORING_PORT", "70000"),
                                     ("LLM_MAX_CONNECTIONS", "0"), ("LLM_PROVIDER", "bogus")])
def test_config_validation_rejects(monkeypatch, var, val):
    monkeypatch.setenv(var, val)
    with pytest.raises(ValueError):
        Config()


def test_config_presets():
    q = Config.from_preset("quality")
    assert q.default_max_tokens == 4096 and q.default_top_p == 0.95
    with pytest.raises(ValueError):
        Config.from_preset("nope")


def test_compute_device_detection(monkeypatch):
    monkeypatch.setenv("COMPUTE_DEVICE", "cpu")
    assert cfgmod._detect_compute_device() == "cpu"
    monkeypatch.setenv("COMPUTE_DEVICE", "rocm")
    monkeypatch.setattr(cfgmod, "_gpu_visible", lambda: True)
    assert cfgmod._detect_compute_device() == "cuda"
    monkeypatch.setattr(cfgmod, "_gpu_visible", lambda: False)
    assert cfgmod._detect_compute_device() == "cpu"


def test_engine_model_resolution(monkeypatch):
    monkeypatch.setenv("LLM_MODEL", "llama3.2:1b")
    monkeypatch.delenv("ENGINE_MODEL", raising=False)
    c = Config()
    assert c.resolved_engine_model() == "llama3.2:1b"
    monkeypatch.setenv("ENGINE_MODEL", "tiny")
    assert Config().current_model() == "tiny"


# ----------------------------------------------------------------------------- logger
def test_structured_logger_respects_level_and_json(tmp_path, capsys):
    log_file = tmp_path / "svc.log"
    lg = StructuredLogger("ft.test.logger", log_level="WARNING", log_file=str(log_file))
    lg.info("hidden")
    lg.warning("shown", session_id="abc")
    request_context.set("req-123456789")
    lg.error("with context")
    request_context.set(None)
    out = capsys.readouterr().out
    assert "hidden" not in out and "shown" in out
    lines = [json.loads(x) for x in log_file.read_text().splitlines()]
    assert lines[0]["message"] == "shown" and lines[0]["session_id"] == "abc"
    assert lines[1]["request_id"] == "req-123456789"
    assert lg.logger.propagate is False


def test_json_formatter_exception():
    rec = logging.LogRecord("x", logging.ERROR, __file__, 1, "boom", None, None)
    doc = json.loads(JsonFormatter().format(rec))
    assert doc["level"] == "ERROR" and doc["message"] == "boom"


# ----------------------------------------------------------------------------- errors
@pytest.mark.parametrize("msg,cat", [
    ("Connection refused by host", ErrorCategory.CONNECTION),
    ("request timed out", ErrorCategory.TIMEOUT),
    ("HIP out of memory on device 0", ErrorCategory.GPU),
    ("at capacity: resource exhausted", ErrorCategory.RESOURCE),
    ("validation failed: bad field", ErrorCategory.VALIDATION),
    ("something odd", ErrorCategory.PROCESSING),
])
def test_error_classification(msg, cat):
    eh = ErrorHandler()
    info = eh.handle_error(RuntimeError(msg))
    assert info.category == cat
    st = eh.get_error_stats()
    assert st["total_errors"] == 1 and st["by_category"][cat.value] == 1
    eh.reset()
    assert eh.get_error_stats()["total_errors"] == 0


def test_service_error_to_dict():
    e = LLMServiceError("nope", category=ErrorCategory.VALIDATION, severity=ErrorSeverity.LOW,
                        recoverable=False)
    d = e.to_dict()
    assert d["message"] == "nope" and d["category"] == "validation" and d["recoverable"] is False
    info = ErrorHandler().handle_error(e, {"session": "s"})
    assert info.category == ErrorCategory.VALIDATION and info.context == {"session": "s"}


def test_circuit_breaker_cycle():
    cb = CircuitBreaker("t", failure_threshold=2, timeout=0.05, half_open_max_calls=1)

    def bad():
        raise RuntimeError("x")

    for _ in range(2):
        with pytest.raises(RuntimeError):
            cb.call(bad)
    assert cb.state == CircuitBreakerState.OPEN
    with pytest.raises(LLMServiceError):
        cb.call(lambda: 1)
    time.sleep(0.06)
    assert cb.call(lambda: 7) == 7  # half-open trial succeeds -> closed
    assert cb.state == CircuitBreakerState.CLOSED


def test_circuit_breaker_async_guard():
    cb = CircuitBreaker("g", failure_threshold=1, timeout=60)

    async def run():
        async with cb.guard():
            pass
        with pytest.raises(ValueError):
            async with cb.guard():
                raise ValueError("bad")
        with pytest.raises(LLMServiceError):
            async with cb.guard():
                pass

    asyncio.run(run())
    assert cb.state == CircuitBreakerState.OPEN
    cb.reset()
    assert cb.state == CircuitBreakerState.CLOSED


def test_retry_with_backoff():
    calls = []

    def flaky():
        calls.append(1)
        if len(calls) < 3:
            raise ConnectionError("again")
        return "ok"

    assert RetryManager.retry_with_backoff(flaky, max_attempts=3, base_delay=0.001) == "ok"
    with pytest.raises(ConnectionError):
        RetryManager.retry_with_backoff(lambda: (_ for _ in ()).throw(ConnectionError("x")),
                                        max_attempts=2, base_delay=0.001)


# ----------------------------------------------------------------------------- connections
def test_connection_manager_limits_and_totals():
    cm = ConnectionManager(max_connections=2)
    assert cm.add_connection("a", object(), {"temperature": 0.5}) is not None
    assert cm.add_connection("b", object()) is not None
    assert cm.add_connection("c", object()) is None  # over the cap
    cm.record_message_received("a")
    cm.record_message_sent("a", 3)
    cm.record_tokens_generated("a", 10)
    cm.record_generation_complete("a")
    cm.record_error("a")
    assert cm.update_config("a", {"max_tokens": 12})
    info = cm.get_connection("a").to_dict()
    assert info["messages_sent"] == 3 and info["config"] == {"temperature": 0.5, "max_tokens": 12}
    assert cm.update_connection_state("a", ConnectionState.PROCESSING)
    assert cm.remove_connection("a") and not cm.remove_connection("a")
    st = cm.get_statistics()
    assert st["active_connections"] == 1 and st["total_tokens_generated"] == 10
    assert st["total_messages_sent"] == 3 and st["total_disconnections"] == 1
    assert st["utilization_percent"] == 50.0
    assert set(cm.get_detailed_stats()["active_sessions"]) == {"b"}
    cm.get_connection("b").last_activity -= 100
    assert cm.cleanup_idle_connections(idle_timeout=50) == 1 and cm.get_active_count() == 0
    cm.reset_statistics()
    assert cm.get_statistics()["total_messages_sent"] == 0


# ----------------------------------------------------------------------------- conversations
def test_conversation_trim_keeps_system_prompt():
    st = ConversationState("s", system_prompt="sys", max_history_length=5)
    st.add_message("system", "sys")
    for i in range(10):
        st.add_message("user" if i % 2 == 0 else "assistant", f"m{i}")
    msgs = st.get_messages_for_api()
    assert len(msgs) == 5 and msgs[0] == {"role": "system", "content": "sys"}
    assert msgs[-1]["content"] == "m9"
    st.clear_history(keep_system_prompt=True)
    assert st.messages == [{"role": "system", "content": "sys"}]
    st.clear_history(keep_system_prompt=False)
    assert st.messages == []


def test_conversation_manager_api():
    cm = ConversationManager(max_history_length=50)
    cm.create_session("s1", system_prompt="be brief")
    assert cm.has_session("s1") and cm.get_session_count() == 1
    assert cm.add_user_message("s1", "hi")
    assert cm.add_assistant_message("s1", "hello", tokens_generated=4)
    assert not cm.add_user_message("missing", "x")
    msgs = cm.get_messages_for_generation("s1")
    assert [m["role"] for m in msgs] == ["system", "user", "assistant"]
    st = cm.get_statistics()
    assert st["active_sessions"] == 1 and st["total_tokens_generated"] == 4 and st["total_turns"] == 3
    assert cm.clear_history("s1") and len(cm.get_messages_for_generation("s1")) == 1
    cm.get_session("s1").last_updated -= 100
    assert cm.cleanup_idle_sessions(idle_timeout=10) == 1 and cm.get_all_session_ids() == []
    assert not cm.end_session("s1")


def test_text_context_and_similarity():
    tc = TextContext()
    head, tail = tc.get_context("Hello there, my friend. How are you?")
    assert head == "Hello there," and tail == " my friend. How are you?"  # 10 alnum chars
    head, _ = tc.get_context("Hi, I am here. Yes", min_alnum_count=8)
    assert head == "Hi, I am here."
    assert tc.get_context("short") == (None, None)
    assert calculate_text_similarity("a b c", "a b d") == pytest.approx(0.5)
    assert calculate_text_similarity("", "x") == 0.0
