"""Model architecture registry (Llama-3 family used by the reference).

Reference model set: ``llama3.2:1b`` (``app/utils/config.py:86``),
``Llama-3.2-3B`` (``docker-compose.vllm.yml:123``), ``Meta-Llama-3.1-8B-Instruct``
(AWQ in ``app/utils/config.py:96``; we run bf16), ``llama3:70b``
(``README.md:474``).  Weights are random-init unless a safetensors checkpoint
directory is given.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Optional


@dataclasses.dataclass(frozen=True)
class ModelConfig:
    name: str
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    vocab_size: int = 128256
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    rms_norm_eps: float = 1e-5
    tie_word_embeddings: bool = False
    max_position_embeddings: int = 8192
    bos_token_id: int = 128000
    eos_token_ids: tuple = (128001, 128008, 128009)

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        h, i, l, v = self.hidden_size, self.intermediate_size, self.num_layers, self.vocab_size
        per_layer = h * (self.q_size + 2 * self.kv_size) + self.q_size * h + 3 * h * i + 2 * h
        emb = v * h * (1 if self.tie_word_embeddings else 2)
        return l * per_layer + emb + h

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes


_LLAMA31_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                    "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}
_LLAMA32_SCALING = {"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                    "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}

MODELS = {
    "llama3.2-1b": ModelConfig("llama3.2-1b", 2048, 16, 32, 8, 64, 8192,
                               rope_scaling=_LLAMA32_SCALING, tie_word_embeddings=True,
                               max_position_embeddings=131072),
    "llama3.2-3b": ModelConfig("llama3.2-3b", 3072, 28, 24, 8, 128, 8192,
                               rope_scaling=_LLAMA32_SCALING, tie_word_embeddings=True,
                               max_position_embeddings=131072),
    "llama3-8b": ModelConfig("llama3-8b", 4096, 32, 32, 8, 128, 14336),
    "llama3.1-8b": ModelConfig("llama3.1-8b", 4096, 32, 32, 8, 128, 14336,
                               rope_scaling=_LLAMA31_SCALING, max_position_embeddings=131072),
    "llama3-70b": ModelConfig("llama3-70b", 8192, 80, 64, 8, 128, 28672),
    "llama3.1-70b": ModelConfig("llama3.1-70b", 8192, 80, 64, 8, 128, 28672,
                                rope_scaling=_LLAMA31_SCALING, max_position_embeddings=131072),
    # 2-layer slices of the real shapes (GPU tests / TP probes: every kernel at its
    # serving shape, a fraction of the weights)
    "llama3-8b-2l": ModelConfig("llama3-8b-2l", 4096, 2, 32, 8, 128, 14336),
    "llama3-70b-2l": ModelConfig("llama3-70b-2l", 8192, 2, 64, 8, 128, 28672),
    # small shapes for CPU tests (keep kernel constraints: hidden % 512 == 0)
    "tiny": ModelConfig("tiny", 512, 2, 8, 2, 64, 1024, vocab_size=128256),
    "tiny-gqa4": ModelConfig("tiny-gqa4", 512, 2, 8, 2, 64, 1536, vocab_size=128256),
    # 8B-shaped heads (d=128, GQA 4) at hidden 2048: exercises the packed-weight decode GEMMs
    "tiny-2k": ModelConfig("tiny-2k", 2048, 2, 16, 4, 128, 4096, vocab_size=128256),
}

# names used by the reference's configuration / Ollama tags / HF ids
ALIASES = {
    "llama3.2:1b": "llama3.2-1b",
    "llama3.2": "llama3.2-3b",
    "llama3.2:3b": "llama3.2-3b",
    "meta-llama/llama-3.2-1b-instruct": "llama3.2-1b",
    "meta-llama/llama-3.2-3b-instruct": "llama3.2-3b",
    "llama3:8b": "llama3-8b",
    "llama3": "llama3-8b",
    "llama-3-8b": "llama3-8b",
    "meta-llama/meta-llama-3-8b-instruct": "llama3-8b",
    "meta-llama/llama-3.1-8b-instruct": "llama3.1-8b",
    "meta-llama/meta-llama-3.1-8b-instruct": "llama3.1-8b",
    "hugging-quants/meta-llama-3.1-8b-instruct-awq-int4": "llama3.1-8b",
    "llama3:70b": "llama3-70b",
    "llama-3-70b": "llama3-70b",
    "meta-llama/meta-llama-3-70b-instruct": "llama3-70b",
    "meta-llama/llama-3.1-70b-instruct": "llama3.1-70b",
}


def resolve_model(name_or_path: str) -> ModelConfig:
    """Resolve a registry name, alias, or a HF checkpoint dir with config.json."""
    key = name_or_path.strip()
    if os.path.isdir(key) and os.path.exists(os.path.join(key, "config.json")):
        return from_hf_config(os.path.join(key, "config.json"))
    low = key.lower()
    if low in MODELS:
        return MODELS[low]
    if low in ALIASES:
        return MODELS[ALIASES[low]]
    raise KeyError(f"unknown model '{name_or_path}'; known: {sorted(MODELS)} + aliases")


def from_hf_config(path: str) -> ModelConfig:
    with open(path) as f:
        c = json.load(f)
    h = c["hidden_size"]
    nh = c["num_attention_heads"]
    eos = c.get("eos_token_id", 128009)
    eos = tuple(eos) if isinstance(eos, list) else (eos,)
    return ModelConfig(
        name=os.path.basename(os.path.dirname(path)) or "hf-model",
        hidden_size=h,
        num_layers=c["num_hidden_layers"],
        num_heads=nh,
        num_kv_heads=c.get("num_key_value_heads", nh),
        head_dim=c.get("head_dim", h // nh),
        intermediate_size=c["intermediate_size"],
        vocab_size=c["vocab_size"],
        rope_theta=c.get("rope_theta", 10000.0),
        rope_scaling=c.get("rope_scaling"),
        rms_norm_eps=c.get("rms_norm_eps", 1e-5),
        tie_word_embeddings=c.get("tie_word_embeddings", False),
        max_position_embeddings=c.get("max_position_embeddings", 8192),
        bos_token_id=c.get("bos_token_id", 128000),
        eos_token_ids=eos,
    )
