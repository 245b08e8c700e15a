"""Engine configuration.

Maps the vLLM engine flags the reference sets in ``docker-compose.vllm.yml:38-53``
(``--max-num-seqs``, ``--max-num-batched-tokens``, ``--max-model-len``,
``--gpu-memory-utilization``, ``--swap-space``, ``--tensor-parallel-size``,
``--dtype``, ``--enforce-eager``) onto our in-process engine.  Existing
``VLLM_*`` env files keep their meaning; ``ENGINE_*`` variables take precedence.
Defaults are sized for one MI355X (288 GB HBM3E): 256 concurrent sequences
instead of vLLM's 32 on a 24 GB card.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Optional, Tuple


def _env(names, default, cast=str):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            try:
                return cast(v)
            except ValueError:
                pass
    return default


def _bool(v: str) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


@dataclasses.dataclass
class EngineConfig:
    model: str = "llama3.1-8b"
    weights: str = "random"            # "random" or a safetensors checkpoint dir
    tokenizer: Optional[str] = None    # tokenizer.json / dir; None -> synthetic Llama-3
    seed: int = 0
    dtype: str = "bfloat16"
    device: str = "auto"               # auto | cuda | cpu
    tp_size: int = 1
    dp_size: int = 1
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    prefill_chunk: int = 512          # soft per-step prefill budget beyond the first prompt (0 = off)
    prefill_chunk_rows: bool = True    # the soft budget also counts the step's decode rows
    guided_prefill_cap: int = 96       # prefill tokens of a step that decodes guided rows (0 = off;
                                       # 96: +0.9 % tok/s on config 5, profiles/ab_guided_cap_r06.txt)
    max_model_len: int = 8192
    gpu_memory_utilization: float = 0.90
    num_kv_blocks: Optional[int] = None
    block_size: int = 16
    swap_space_gb: float = 4.0
    enable_prefix_caching: bool = True
    enforce_eager: bool = False        # disable hipGraph decode capture
    graph_batch_sizes: Tuple[int, ...] = (1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 128, 160, 192, 224, 256)
    async_output: bool = True          # overlap detokenize/streaming with the next GPU step
    pipeline_depth: int = 1            # decode steps queued on the GPU ahead of the one collected
    separate_process: bool = False     # run the step loop in its own process (no GIL sharing)
    # TP: xGMI one/two-shot all-reduce (and the fused all-reduce + add + RMSNorm) for
    # decode-size messages, RCCL above; on by default, falls back to RCCL when the IPC
    # mapping fails or a peer times out
    custom_allreduce: bool = True
    tp_share_device: bool = False      # TP ranks all on device_base (tests: gloo control + IPC data)
    max_restarts: int = 3              # separate-process engines: respawns after a replica dies
    quantization: Optional[str] = None  # None | "awq" | "w4" (W4A16, group 128; --quantization awq)
    # a sequence's tokens independent of what else shares its steps (fixed GEMM splits,
    # fixed-piece attention partitions; TP=1, bf16; slower decode attention)
    batch_invariant: bool = False
    # KV-cache storage: "auto" (the compute dtype) | "fp8" (OCP e4m3 at scale 1, vLLM's
    # --kv-cache-dtype fp8 without calibration): half the cache bytes per token, so the
    # decode attention stream halves and the pool holds twice the tokens
    kv_cache_dtype: str = "auto"

    def kv_torch_dtype(self, compute_dtype):
        import torch

        v = (self.kv_cache_dtype or "auto").lower()
        if v in ("auto", "bf16", "bfloat16", "float32", "fp32"):
            return compute_dtype
        if v in ("fp8", "fp8_e4m3", "float8_e4m3fn", "e4m3"):
            return torch.float8_e4m3fn
        raise ValueError(f"kv_cache_dtype {self.kv_cache_dtype!r}: auto | fp8")

    def resolved_device(self) -> str:
        if self.device != "auto":
            return self.device
        try:
            import torch

            return "cuda" if torch.cuda.is_available() else "cpu"
        except Exception:
            return "cpu"

    def torch_dtype(self):
        import torch

        if self.resolved_device() == "cpu" and self.dtype in ("auto", "bfloat16") and \
                os.environ.get("ENGINE_CPU_BF16", "0") != "1":
            return torch.float32  # CPU backend computes in fp32
        return {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float16": torch.bfloat16,
                "half": torch.bfloat16, "auto": torch.bfloat16,
                "float32": torch.float32}[self.dtype]

    @classmethod
    def from_env(cls, model: Optional[str] = None, **overrides) -> "EngineConfig":
        c = cls(
            model=model or _env(["ENGINE_MODEL", "VLLM_MODEL"], cls.model),
            weights=_env(["ENGINE_WEIGHTS", "MODEL_WEIGHTS"], "random"),
            tokenizer=_env(["ENGINE_TOKENIZER"], None),
            seed=_env(["ENGINE_SEED"], 0, int),
            dtype=_env(["ENGINE_DTYPE", "VLLM_DTYPE"], "bfloat16"),
            device=_env(["ENGINE_DEVICE"], "auto"),
            tp_size=_env(["ENGINE_TP_SIZE", "VLLM_TENSOR_PARALLEL_SIZE"], 1, int),
            dp_size=_env(["ENGINE_DP_SIZE"], 1, int),
            max_num_seqs=_env(["ENGINE_MAX_NUM_SEQS", "VLLM_MAX_NUM_SEQS"], 256, int),
            max_num_batched_tokens=_env(["ENGINE_MAX_NUM_BATCHED_TOKENS",
                                         "VLLM_MAX_NUM_BATCHED_TOKENS"], 8192, int),
            max_model_len=_env(["ENGINE_MAX_MODEL_LEN", "VLLM_MAX_MODEL_LEN"], 8192, int),
            prefill_chunk=_env(["ENGINE_PREFILL_CHUNK"], 512, int),
            prefill_chunk_rows=_env(["ENGINE_PREFILL_CHUNK_ROWS"], "1", str).lower() in ("1", "true"),
            guided_prefill_cap=_env(["ENGINE_GUIDED_PREFILL_CAP"], 96, int),
            gpu_memory_utilization=_env(["ENGINE_GPU_MEMORY_UTILIZATION",
                                         "VLLM_GPU_MEMORY_UTILIZATION"], 0.90, float),
            num_kv_blocks=_env(["ENGINE_NUM_KV_BLOCKS"], None, int),
            block_size=_env(["ENGINE_BLOCK_SIZE"], 16, int),
            swap_space_gb=_env(["ENGINE_SWAP_SPACE", "VLLM_SWAP_SPACE"], 4.0, float),
            enable_prefix_caching=_env(["ENGINE_PREFIX_CACHING"], True, _bool),
            enforce_eager=_env(["ENGINE_ENFORCE_EAGER", "VLLM_ENFORCE_EAGER"], False, _bool),
            separate_process=_env(["ENGINE_SEPARATE_PROCESS"], None, _bool),
            pipeline_depth=max(1, min(3, _env(["ENGINE_PIPELINE_DEPTH"], 1, int))),
            custom_allreduce=_env(["ENGINE_CUSTOM_ALLREDUCE"], True, _bool),
            tp_share_device=_env(["ENGINE_TP_SHARE_DEVICE"], False, _bool),
            max_restarts=_env(["ENGINE_MAX_RESTARTS"], 3, int),
            quantization=_env(["ENGINE_QUANTIZATION", "VLLM_QUANTIZATION"], None) or None,
            batch_invariant=_env(["ENGINE_BATCH_INVARIANT", "VLLM_BATCH_INVARIANT"], False, _bool),
            kv_cache_dtype=_env(["ENGINE_KV_CACHE_DTYPE", "VLLM_KV_CACHE_DTYPE"], "auto"),
        )
        for k, v in overrides.items():
            setattr(c, k, v)
        if c.separate_process is None:
            # a TP group runs in its own process by default: when a worker dies the
            # supervisor (parallel/dp_router.py) can tear the group down and respawn it
            c.separate_process = c.tp_size > 1
        if c.quantization is None and "awq" in c.model.lower():
            # the reference's default model (hugging-quants/...-AWQ-INT4) runs W4A16
            c.quantization = "awq"
        return c
