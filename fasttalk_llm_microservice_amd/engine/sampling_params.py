"""Sampling parameters (E10).  Mirrors what the reference forwards to its
backends: temperature / max_tokens / top_p / stop (vLLM,
``app/core/vllm_handler.py:149-164``) and top_k / num_predict (Ollama,
``app/core/ollama_handler.py:145-155``)."""
from __future__ import annotations

import dataclasses
import random
from typing import Any, List, Optional


@dataclasses.dataclass
class SamplingParams:
    temperature: float = 0.7
    top_p: float = 1.0
    top_k: int = 0               # <= 0: disabled
    max_tokens: int = 2048
    min_tokens: int = 0
    stop: Optional[List[str]] = None
    stop_token_ids: Optional[List[int]] = None
    ignore_eos: bool = False
    seed: Optional[int] = None
    guided: Any = None           # engine.guided.GuidedSpec (JSON-schema constrained decoding)
    # the grammar binds only if the first generated token is a valid start of it (e.g.
    # the model chose to open a tool call with '{"'); otherwise the reply is free text
    guided_lazy: bool = False
    skip_special_tokens: bool = True
    # scheduling priority: waiting prompts of a higher priority are prefilled first
    # (an agent's post-tool re-prompt: its user has already waited through the call)
    priority: int = 0

    def __post_init__(self):
        if self.temperature is None:
            self.temperature = 0.7
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if self.top_p is None:
            self.top_p = 1.0
        if not 0.0 < self.top_p <= 1.0:
            raise ValueError("top_p must be in (0, 1]")
        if self.top_k is None:
            self.top_k = 0
        if self.max_tokens is None or self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if self.seed is None:
            self.seed = random.getrandbits(62)
        if isinstance(self.stop, str):
            self.stop = [self.stop]
