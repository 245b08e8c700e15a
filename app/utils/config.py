"""Service configuration (env -> dataclass), API-compatible with the reference
``app/utils/config.py`` (``Config`` fields, env names and defaults of Appendix C,
``to_dict``, ``from_preset``, ``get_config``).

Differences:
* provider ``native`` (the in-process MI355X engine) is valid and is the
  default; ``vllm`` / ``ollama`` / ``openai`` remain remote providers (Q20:
  ``openai`` = any OpenAI-compatible base URL).
* ``COMPUTE_DEVICE`` drives the engine device (Q21): ``cuda``/``rocm``/``hip``
  -> the GPU (ROCm torch exposes it as ``cuda``), ``cpu`` -> reference ops.
* engine knobs (``ENGINE_*``, and the compose-level ``VLLM_*`` engine flags) are
  surfaced here so ``python main.py config --show`` prints them.
"""
from __future__ import annotations

import logging
import os
import sys
from dataclasses import dataclass, field
from typing import Any, Dict

logger = logging.getLogger(__name__)

VALID_PROVIDERS = ("native", "vllm", "ollama", "openai")
DEFAULT_SYSTEM_PROMPT = "You are a helpful voice assistant. Keep responses concise and conversational."


def _e(name: str, default: str) -> str:
    v = os.getenv(name)
    return default if v is None else v


def _flag(name: str, default: str = "true") -> bool:
    return _e(name, default).strip().lower() == "true"


def _gpu_visible() -> bool:
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                "NVIDIA_VISIBLE_DEVICES"):
        if os.getenv(var):
            return True
    return os.path.exists("/dev/kfd")


def _detect_compute_device() -> str:
    """``cuda`` (any ROCm/HIP GPU), ``cpu`` or ``mps``; explicit COMPUTE_DEVICE wins."""
    want = os.getenv("COMPUTE_DEVICE", "").strip().lower()
    if want in ("rocm", "hip", "gpu"):
        want = "cuda"
    if want == "cpu":
        return "cpu"
    if want == "mps":
        if sys.platform == "darwin":
            return "mps"
        logger.warning("MPS requested but not on macOS; using CPU")
        return "cpu"
    if want == "cuda":
        if _gpu_visible():
            return "cuda"
        logger.warning("GPU requested but no GPU is visible; using CPU")
        return "cpu"
    if _gpu_visible():
        return "cuda"
    return "mps" if sys.platform == "darwin" else "cpu"


@dataclass
class Config:
    # ---- compute device
    compute_device: str = field(default_factory=_detect_compute_device)
    # ---- provider / model
    llm_provider: str = field(default_factory=lambda: _e("LLM_PROVIDER", "native"))
    model_name: str = field(default_factory=lambda: _e("LLM_MODEL", "llama3.2:1b"))
    device: str = field(default_factory=_detect_compute_device)  # legacy alias
    # ---- remote OpenAI-compatible backend (vLLM)
    vllm_base_url: str = field(default_factory=lambda: _e("VLLM_BASE_URL", "http://vllm:8000/v1"))
    vllm_model: str = field(default_factory=lambda: _e(
        "VLLM_MODEL", "hugging-quants/Meta-Llama-3.1-8B-Instruct-AWQ-INT4"))
    vllm_api_key: str = field(default_factory=lambda: _e("VLLM_API_KEY", "not-needed"))
    vllm_timeout: float = field(default_factory=lambda: float(_e("VLLM_TIMEOUT", "600.0")))
    # ---- agent
    enable_pydantic_ai: bool = field(default_factory=lambda: _flag("ENABLE_PYDANTIC_AI"))
    enable_web_search: bool = field(default_factory=lambda: _flag("ENABLE_WEB_SEARCH"))
    enable_tools: bool = field(default_factory=lambda: _flag("ENABLE_TOOLS"))
    duckduckgo_rate_limit: float = field(default_factory=lambda: float(_e("DUCKDUCKGO_RATE_LIMIT", "1.0")))
    system_prompt: str = field(default_factory=lambda: _e("SYSTEM_PROMPT", DEFAULT_SYSTEM_PROMPT))
    # ---- remote Ollama backend
    ollama_base_url: str = field(default_factory=lambda: _e("OLLAMA_BASE_URL", "http://ollama:11434"))
    ollama_keep_alive: str = field(default_factory=lambda: _e("OLLAMA_KEEP_ALIVE", "5m"))
    ollama_timeout: float = field(default_factory=lambda: float(_e("OLLAMA_TIMEOUT", "600.0")))
    # ---- generation defaults
    default_temperature: float = field(default_factory=lambda: float(_e("DEFAULT_TEMPERATURE", "0.7")))
    default_max_tokens: int = field(default_factory=lambda: int(_e("DEFAULT_MAX_TOKENS", "2048")))
    default_context_window: int = field(default_factory=lambda: int(_e("DEFAULT_CONTEXT_WINDOW", "8192")))
    default_top_p: float = field(default_factory=lambda: float(_e("DEFAULT_TOP_P", "0.9")))
    default_top_k: int = field(default_factory=lambda: int(_e("DEFAULT_TOP_K", "40")))
    # ---- server
    host: str = field(default_factory=lambda: _e("LLM_HOST", "0.0.0.0"))
    port: int = field(default_factory=lambda: int(_e("LLM_PORT", "8000")))
    max_connections: int = field(default_factory=lambda: int(_e("LLM_MAX_CONNECTIONS", "50")))
    log_level: str = field(default_factory=lambda: _e("LOG_LEVEL", "INFO"))
    # ---- monitoring
    monitoring_port: int = field(default_factory=lambda: int(_e("LLM_MONITORING_PORT", "9092")))
    monitoring_host: str = field(default_factory=lambda: _e("LLM_MONITORING_HOST", "0.0.0.0"))
    # ---- performance (kept for compatibility; the engine sizes itself)
    num_threads: int = field(default_factory=lambda: int(_e("NUM_THREADS", "12")))
    num_workers: int = field(default_factory=lambda: int(_e("NUM_WORKERS", "6")))
    # ---- sessions
    session_timeout: int = field(default_factory=lambda: int(_e("SESSION_TIMEOUT", "3600")))
    max_history_length: int = field(default_factory=lambda: int(_e("MAX_HISTORY_LENGTH", "50")))
    # ---- paths
    model_path: str = field(default_factory=lambda: _e("MODEL_PATH", "/app/models"))
    log_path: str = field(default_factory=lambda: _e("LOG_PATH", "/app/logs"))
    # ---- in-process MI355X engine (provider "native")
    engine_model: str = field(default_factory=lambda: _e("ENGINE_MODEL", ""))
    engine_weights: str = field(default_factory=lambda: _e("ENGINE_WEIGHTS", "random"))
    engine_tp_size: int = field(default_factory=lambda: int(_e(
        "ENGINE_TP_SIZE", _e("VLLM_TENSOR_PARALLEL_SIZE", "1"))))
    engine_dp_size: int = field(default_factory=lambda: int(_e("ENGINE_DP_SIZE", "1")))
    # DP>1: "workers" = N service processes on one port (SO_REUSEPORT, app/server/workers.py);
    # "router" = one service process in front of N engine replica processes
    engine_dp_mode: str = field(default_factory=lambda: _e("ENGINE_DP_MODE", "workers").lower())
    engine_max_num_seqs: int = field(default_factory=lambda: int(_e(
        "ENGINE_MAX_NUM_SEQS", _e("VLLM_MAX_NUM_SEQS", "256"))))
    engine_max_model_len: int = field(default_factory=lambda: int(_e(
        "ENGINE_MAX_MODEL_LEN", _e("VLLM_MAX_MODEL_LEN", "8192"))))
    engine_gpu_memory_utilization: float = field(default_factory=lambda: float(_e(
        "ENGINE_GPU_MEMORY_UTILIZATION", _e("VLLM_GPU_MEMORY_UTILIZATION", "0.90"))))
    # opt-in: decode agent tool calls under the JSON-schema token FSM when the user
    # message asks for search / time / session info (BASELINE config 5)
    agent_json_tool_calls: bool = field(default_factory=lambda: _flag("AGENT_GUIDED_TOOL_CALLS", "false"))

    def __post_init__(self):
        self._validate()
        self._log_config()

    # ------------------------------------------------------------------ checks
    def _validate(self):
        if not (0.0 <= self.default_temperature <= 2.0):
            logger.warning("Temperature %s is outside recommended range [0.0, 2.0]",
                           self.default_temperature)
        problems = [
            (0.0 <= self.default_top_p <= 1.0, f"top_p must be between 0.0 and 1.0, got {self.default_top_p}"),
            (self.default_top_k >= 1, f"top_k must be >= 1, got {self.default_top_k}"),
            (self.default_max_tokens >= 1, f"max_tokens must be >= 1, got {self.default_max_tokens}"),
            (1024 <= self.port <= 65535, f"Port must be between 1024 and 65535, got {self.port}"),
            (1024 <= self.monitoring_port <= 65535,
             f"Monitoring port must be between 1024 and 65535, got {self.monitoring_port}"),
            (self.max_connections >= 1, f"max_connections must be >= 1, got {self.max_connections}"),
            (self.llm_provider in VALID_PROVIDERS,
             f"llm_provider must be one of {VALID_PROVIDERS}, got {self.llm_provider}"),
        ]
        for ok, msg in problems:
            if not ok:
                raise ValueError(msg)
        if self.default_context_window < self.default_max_tokens:
            logger.warning("Context window (%s) is smaller than max_tokens (%s)",
                           self.default_context_window, self.default_max_tokens)

    def _log_config(self):
        lines = [f"LLM Provider: {self.llm_provider}", f"Compute Device: {self.compute_device}"]
        if self.llm_provider == "native":
            lines += [f"Engine Model: {self.resolved_engine_model()}",
                      f"Engine Weights: {self.engine_weights}",
                      f"Tensor Parallel: {self.engine_tp_size}  Data Parallel: {self.engine_dp_size}"]
        elif self.llm_provider in ("vllm", "openai"):
            lines += [f"vLLM Model: {self.vllm_model}", f"vLLM URL: {self.vllm_base_url}",
                      f"PydanticAI Enabled: {self.enable_pydantic_ai}"]
        else:
            lines += [f"Model: {self.model_name}", f"Ollama URL: {self.ollama_base_url}"]
        lines += [f"Server: {self.host}:{self.port}",
                  f"Monitoring: {self.monitoring_host}:{self.monitoring_port}",
                  f"Max Connections: {self.max_connections}",
                  f"Temperature: {self.default_temperature}  Max Tokens: {self.default_max_tokens}",
                  f"Context Window: {self.default_context_window}", f"Log Level: {self.log_level}"]
        for line in lines:
            logger.info(line)

    # ------------------------------------------------------------------ helpers
    def resolved_engine_model(self) -> str:
        """Model the native engine serves: ENGINE_MODEL, else the configured tag."""
        if self.engine_model:
            return self.engine_model
        return self.model_name if self.llm_provider in ("native", "ollama") else self.vllm_model

    def current_model(self) -> str:
        if self.llm_provider in ("vllm", "openai"):
            return self.vllm_model
        if self.llm_provider == "native":
            return self.resolved_engine_model()
        return self.model_name

    def to_dict(self) -> Dict[str, Any]:
        keys = ["llm_provider", "compute_device", "model_name", "device", "host", "port",
                "monitoring_port", "max_connections", "default_temperature", "default_max_tokens",
                "default_context_window", "default_top_p", "default_top_k", "num_threads",
                "num_workers", "log_level"]
        d: Dict[str, Any] = {k: getattr(self, k) for k in keys}
        if self.llm_provider in ("vllm", "openai"):
            extra = ["vllm_base_url", "vllm_model", "enable_pydantic_ai", "enable_web_search",
                     "enable_tools"]
        elif self.llm_provider == "native":
            extra = ["engine_weights", "engine_tp_size", "engine_dp_size", "engine_max_num_seqs",
                     "engine_max_model_len", "engine_gpu_memory_utilization", "enable_pydantic_ai",
                     "enable_web_search", "enable_tools"]
            d["engine_model"] = self.resolved_engine_model()
        else:
            extra = ["ollama_base_url", "ollama_keep_alive"]
        d.update({k: getattr(self, k) for k in extra})
        return d

    PRESETS = {
        "fast": dict(default_temperature=0.5, default_max_tokens=1024, default_context_window=4096,
                     default_top_p=0.9, default_top_k=40),
        "balanced": dict(default_temperature=0.7, default_max_tokens=2048,
                         default_context_window=8192, default_top_p=0.9, default_top_k=40),
        "quality": dict(default_temperature=0.8, default_max_tokens=4096,
                        default_context_window=16384, default_top_p=0.95, default_top_k=50),
    }

    @classmethod
    def from_preset(cls, preset: str) -> "Config":
        if preset not in cls.PRESETS:
            raise ValueError(f"Unknown preset '{preset}'. Choose from: {list(cls.PRESETS)}")
        cfg = cls()
        for k, v in cls.PRESETS[preset].items():
            setattr(cfg, k, v)
        return cfg


def get_config() -> Config:
    return Config()
