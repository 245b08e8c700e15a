"""FastTalk LLM microservice on AMD Instinct MI355X.

WebSocket token streaming (``/ws/llm``) with per-session conversation history,
served from an in-process inference engine (package
``fasttalk_llm_microservice_amd``: hand-written gfx950 HIP kernels, paged KV
cache, continuous batching, hipGraph decode, RCCL tensor parallelism).
Public import surface kept from the reference (``app/__init__.py:19-25``).
"""

__version__ = "1.0.0"
__author__ = "FastTalk Team"

from app.utils.config import Config  # noqa: E402
from app.utils.logger import StructuredLogger  # noqa: E402

__all__ = ["Config", "StructuredLogger"]
