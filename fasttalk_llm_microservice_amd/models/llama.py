"""Llama-3 decoder for the in-process engine (replaces the vLLM container the
reference talks to over HTTP: ``app/core/vllm_handler.py:53-62``).

Per layer:  fused add+RMSNorm (K2, HIP) -> QKV GEMM (K3,
hipBLASLt) -> RoPE + paged KV write (K4, HIP) -> prefill flash attention (K5,
HIP/MFMA) or paged split-K decode attention (K6, HIP) -> O GEMM (K7) [+ RCCL
all-reduce under TP] -> fused add+RMSNorm -> gate_up GEMM (K8) -> SiLU-mul
(K9, HIP) -> down GEMM (K10) [+ all-reduce].  Only the last-token rows reach the
final norm and the LM head (K11), and the sampler (K12) consumes bf16 logits
directly.  The same code runs the CPU backend through the fp32 reference ops.
"""
from __future__ import annotations

import dataclasses
import os
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import reference as ref
from ..parallel.comm import SINGLE, TPComm
from .config import ModelConfig
from . import weights as W


@dataclasses.dataclass
class AttnMeta:
    """Per-step attention metadata (device tensors, int32).

    Rows ``[0, num_decode)`` are decode rows (one new token per sequence, paged
    split-K decode kernel); rows ``[num_decode, T)`` are prefill chunks (varlen
    MFMA prefill kernel).  A step may contain either or both (mixed batching).
    """
    positions: torch.Tensor          # [T]
    slot_mapping: torch.Tensor       # [T]
    logits_indices: torch.Tensor     # [B] rows that need logits (int64)
    num_decode: int = 0
    # decode rows
    dec_block_tables: Optional[torch.Tensor] = None   # [num_decode, max_blocks]
    dec_seq_lens: Optional[torch.Tensor] = None       # [num_decode]
    max_splits: int = 1
    tmp_out: Optional[torch.Tensor] = None
    tmp_ml: Optional[torch.Tensor] = None
    # prefill rows
    block_tables: Optional[torch.Tensor] = None       # [P, max_blocks]
    seq_lens: Optional[torch.Tensor] = None           # [P] kv length after this step
    q_start_loc: Optional[torch.Tensor] = None        # [P+1], relative to row num_decode
    tile_info: Optional[torch.Tensor] = None          # [num_tiles*2]
    num_tiles: int = 0

    @property
    def is_prefill(self) -> bool:
        return self.num_decode == 0


@dataclasses.dataclass
class LayerWeights:
    wqkv: torch.Tensor
    wo: torch.Tensor
    wgu: torch.Tensor
    wd: torch.Tensor
    ln1: torch.Tensor
    ln2: torch.Tensor
    wd_pk: Optional[torch.Tensor] = None   # down proj in the MFMA-fragment image (decode GEMM)
    wgu_pk: Optional[torch.Tensor] = None  # gate_up in the MFMA-fragment image


# decode (<= 64 rows) GEMMs on pre-packed weights, measured from cold caches on
# MI355X at M = 64 (bench/gemm_sweep.py): down 28 us vs hipBLASLt 40 us, gate_up
# 46 vs 55, LM head 197 vs 212.  The down projection runs split-K into fp32 slabs
# that the next residual-add + RMSNorm reduces (no extra kernel); gate_up's two
# slabs are reduced by the SiLU-mul kernel (which runs anyway); the LM head
# stores bf16.
DOWN_SPLITS = 4
GU_SPLITS = 2
PACKED_ROWS = 64


class LlamaModel:
    def __init__(self, cfg: ModelConfig, device: torch.device, dtype: torch.dtype = torch.bfloat16,
                 comm: TPComm = SINGLE, max_model_len: int = 8192):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.comm = comm
        self.tp = comm.world_size
        self.rank = comm.rank
        self.nq, self.nkv = W.tp_heads(cfg, self.tp)
        self.d = cfg.head_dim
        self.scale = self.d ** -0.5
        self.vocab_shard = cfg.vocab_size // self.tp
        assert cfg.vocab_size % self.tp == 0
        self.max_model_len = max_model_len
        self.layers: List[LayerWeights] = []
        self.embed: Optional[torch.Tensor] = None
        self.norm: Optional[torch.Tensor] = None
        self.lm_head: Optional[torch.Tensor] = None
        self.cos_sin = ref.rope_cos_sin(self.d, max(max_model_len, 16) + 1, cfg.rope_theta,
                                        cfg.rope_scaling, device=self.device)
        self.lm_head_pk: Optional[torch.Tensor] = None
        self.ws: Optional[torch.Tensor] = None
        self.use_packed = (self.device.type == "cuda" and dtype == torch.bfloat16
                           and os.environ.get("FT_PACKED_GEMM", "1") != "0")

    # ------------------------------------------------------------------ weights
    def _set_layers(self, shards):
        self.layers = [LayerWeights(**{k: v.to(self.device, self.dtype) for k, v in s.items()})
                       for s in shards]

    def init_random(self, seed: int = 0, std: float = 0.02, consistent: Optional[bool] = None):
        """Random-init weights.  ``consistent`` (default: small models) draws the
        full unsharded tensors on the host from one seed and slices them, so TP=N
        equals TP=1 exactly; otherwise every shard is drawn on the device."""
        cfg = self.cfg
        if consistent is None:
            consistent = cfg.num_params() < 2_000_000_000 and self.device.type == "cpu" or \
                cfg.num_params() < 300_000_000
        if consistent:
            g = torch.Generator().manual_seed(seed)
            embed = (torch.randn(cfg.vocab_size, cfg.hidden_size, generator=g) * std).to(self.dtype)
            shards = []
            for li in range(cfg.num_layers):
                full = W.random_full_layer(cfg, g, std, self.dtype)
                shards.append(W.shard_full_layer(cfg, full, self.rank, self.tp))
            self._set_layers(shards)
            lm = embed if cfg.tie_word_embeddings else \
                (torch.randn(cfg.vocab_size, cfg.hidden_size, generator=g) * std).to(self.dtype)
            self.embed = embed.to(self.device)
            self.lm_head = W._shard_rows(lm, self.rank, self.tp).contiguous().to(self.device)
        else:
            self.layers = []
            for li in range(cfg.num_layers):
                s = W.random_layer_fast(cfg, self.rank, self.tp, li, seed, std, self.dtype, self.device)
                self.layers.append(LayerWeights(**s))
            g = torch.Generator(device=self.device)
            g.manual_seed(seed * 7 + 3)
            self.embed = torch.empty(cfg.vocab_size, cfg.hidden_size, dtype=self.dtype,
                                     device=self.device).normal_(0.0, std, generator=g)
            if cfg.tie_word_embeddings:
                self.lm_head = W._shard_rows(self.embed, self.rank, self.tp)
            else:
                self.lm_head = torch.empty(self.vocab_shard, cfg.hidden_size, dtype=self.dtype,
                                           device=self.device).normal_(0.0, std, generator=g)
        self.norm = torch.ones(cfg.hidden_size, dtype=self.dtype, device=self.device)
        self._prepare_packed()
        return self

    def load_checkpoint(self, ckpt_dir: str):
        cfg = self.cfg
        idx = W.SafetensorsIndex(ckpt_dir)
        shards = []
        for li in range(cfg.num_layers):
            full = W.load_full_layer(idx, li, self.dtype)
            shards.append(W.shard_full_layer(cfg, full, self.rank, self.tp))
        self._set_layers(shards)
        self.embed = idx.get("model.embed_tokens.weight").to(self.device, self.dtype)
        self.norm = idx.get("model.norm.weight").to(self.device, self.dtype)
        if cfg.tie_word_embeddings or not idx.has("lm_head.weight"):
            lm = self.embed
        else:
            lm = idx.get("lm_head.weight").to(self.dtype)
        self.lm_head = W._shard_rows(lm, self.rank, self.tp).contiguous().to(self.device)
        self._prepare_packed()
        return self

    def _prepare_packed(self):
        """Adds the packed copies the decode GEMMs stream (one extra copy of the
        down projections and the LM head: ~4 GB for Llama-3-8B, of 288 GB)."""
        if not self.use_packed:
            return
        cfg = self.cfg
        H = cfg.hidden_size
        inter = self.layers[0].wd.shape[1] if self.layers else 0
        down_ok = (self.tp == 1 and H % 2048 == 0 and H % 64 == 0
                   and inter % (64 * DOWN_SPLITS) == 0)
        # gate_up on packed weights measured no faster in the serving loop than
        # hipBLASLt (the slab reduction eats the GEMM gain) and costs another
        # copy of the largest weight: opt-in
        gu_ok = (down_ok and H % (512 * GU_SPLITS) == 0 and (2 * inter) % 32 == 0
                 and os.environ.get("FT_PACKED_GATE_UP", "0") == "1")
        for L in self.layers:
            L.wd_pk = ops.pack_weight(L.wd) if down_ok else None
            L.wgu_pk = ops.pack_weight(L.wgu) if gu_ok else None
        if self.lm_head is not None and self.lm_head.shape[0] % 32 == 0 and H % 512 == 0:
            self.lm_head_pk = ops.pack_weight(self.lm_head)
        if down_ok:
            n = max(DOWN_SPLITS * H, GU_SPLITS * 2 * inter if gu_ok else 0)
            self.ws = torch.empty(PACKED_ROWS * n, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------------ KV cache
    def kv_cache_shape(self, num_blocks: int, block_size: int) -> Tuple[int, ...]:
        return (num_blocks, self.nkv, block_size, self.d)

    def allocate_kv_cache(self, num_blocks: int, block_size: int):
        shp = self.kv_cache_shape(num_blocks, block_size)
        return [(torch.zeros(shp, dtype=self.dtype, device=self.device),
                 torch.zeros(shp, dtype=self.dtype, device=self.device))
                for _ in range(self.cfg.num_layers)]

    # ------------------------------------------------------------------ forward
    def forward(self, input_ids: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """Returns the final-normed hidden rows at ``meta.logits_indices``."""
        cfg = self.cfg
        eps = cfg.rms_norm_eps
        nq, nkv, d = self.nq, self.nkv, self.d
        t = input_ids.shape[0]
        H = cfg.hidden_size
        residual = None
        x = None
        slab = False  # the previous down projection left fp32 split-K slabs in self.ws
        packed = t <= PACKED_ROWS and self.ws is not None
        for li, L in enumerate(self.layers):
            if residual is None:
                x, residual = ops.embed_rmsnorm(input_ids, self.embed, L.ln1, eps)  # K1 + K2
            elif slab:  # residual += sum(slabs); x = rmsnorm(residual) * ln1
                x = torch.empty(t, H, dtype=self.dtype, device=self.device)
                ops.row_rmsnorm(x, L.ln1, eps, t, ws=self.ws, splits=DOWN_SPLITS, residual=residual)
                slab = False
            else:
                ops.fused_add_rmsnorm(x, residual, L.ln1, eps)
            qkv = F.linear(x, L.wqkv)
            kc, vc = kv_caches[li]
            ops.rope_kv_write(qkv, meta.positions, self.cos_sin, meta.slot_mapping, kc, vc, nq, nkv, d)
            attn = torch.empty(t, nq * d, dtype=x.dtype, device=x.device)
            nd = meta.num_decode
            if nd > 0:
                ops.decode_attention(attn[:nd], qkv[:nd], kc, vc, meta.dec_block_tables,
                                     meta.dec_seq_lens, meta.tmp_out, meta.tmp_ml, nq, nkv, d,
                                     meta.max_splits, self.scale)
            if t > nd:
                ops.prefill_attention(attn[nd:], qkv[nd:], kc, vc, meta.block_tables, meta.seq_lens,
                                      meta.q_start_loc, meta.tile_info, meta.num_tiles, nq, nkv, d,
                                      self.scale)
            x = F.linear(attn, L.wo)
            self.comm.all_reduce(x)
            ops.fused_add_rmsnorm(x, residual, L.ln2, eps)
            if packed and L.wgu_pk is not None:
                ops.skinny_gemm(x, L.wgu_pk, ws=self.ws, splits=GU_SPLITS, nt=2, u=-4)
                inter = L.wgu.shape[0] // 2
                h = torch.empty(t, inter, dtype=self.dtype, device=self.device)
                ops.slab_silu(self.ws, GU_SPLITS, t, inter, h)
            else:
                gu = F.linear(x, L.wgu)
                h = ops.silu_mul(gu)
            if packed and L.wd_pk is not None:
                ops.skinny_gemm(h, L.wd_pk, ws=self.ws, splits=DOWN_SPLITS, nt=4, u=-3)
                slab = True
            else:
                x = F.linear(h, L.wd)
                self.comm.all_reduce(x)
        if slab:
            x = torch.empty(t, H, dtype=self.dtype, device=self.device)
            ops.slab_store(self.ws, DOWN_SPLITS, t, H, x)
        idx = meta.logits_indices
        if idx.numel() != t:
            x = x.index_select(0, idx)
            residual = residual.index_select(0, idx)
        else:
            residual = residual.clone()
        ops.fused_add_rmsnorm(x, residual, self.norm, eps)
        return x

    def compute_logits(self, h: torch.Tensor) -> torch.Tensor:
        """[B, H] -> [B, V] logits (bf16 on GPU; vocab-parallel shards gathered)."""
        if self.lm_head_pk is not None and h.shape[0] <= PACKED_ROWS:
            logits = torch.empty(h.shape[0], self.lm_head.shape[0], dtype=h.dtype, device=h.device)
            ops.skinny_gemm(h, self.lm_head_pk, out=logits, splits=1, nt=2, u=-4)
        else:
            logits = F.linear(h, self.lm_head)
        return self.comm.all_gather_last(logits)
