"""Weights: deterministic random init and (TP-sharded) safetensors loading.

Layout produced here and handed to :class:`LlamaModel` (all
``[out_features, in_features]``; on the GPU the model re-lays every projection out
into the MFMA-fragment image the hand-written GEMMs stream, ``ops.pack_weight``, and
drops these row-major tensors; the CPU backend keeps them for ``F.linear``):

* ``wqkv``  [ (nq + 2 nkv)/tp * D, H ]   column parallel, q|k|v fused
* ``wo``    [ H, nq/tp * D ]             row parallel (all-reduce after)
* ``wgu``   [ 2 I/tp, H ]                column parallel, gate|up fused
* ``wd``    [ H, I/tp ]                  row parallel (all-reduce after)
* ``embed`` [ V, H ] replicated; ``lm_head`` [ V/tp, H ] vocab parallel.

E14 in SURVEY.md §2.3 (model weights cache -> random-init or local checkpoint).
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, Optional

import torch

from .config import ModelConfig


def tp_heads(cfg: ModelConfig, tp: int):
    assert cfg.num_heads % tp == 0, "num_heads must divide by tp"
    nq = cfg.num_heads // tp
    if cfg.num_kv_heads >= tp:
        assert cfg.num_kv_heads % tp == 0
        nkv = cfg.num_kv_heads // tp
    else:
        assert tp % cfg.num_kv_heads == 0
        nkv = 1
    return nq, nkv


def kv_head_range(cfg: ModelConfig, tp: int, rank: int):
    nq, nkv = tp_heads(cfg, tp)
    if cfg.num_kv_heads >= tp:
        return rank * nkv, (rank + 1) * nkv
    rep = tp // cfg.num_kv_heads
    h = rank // rep
    return h, h + 1


def _shard_rows(t: torch.Tensor, rank: int, tp: int) -> torch.Tensor:
    n = t.shape[0] // tp
    return t[rank * n:(rank + 1) * n]


def _shard_cols(t: torch.Tensor, rank: int, tp: int) -> torch.Tensor:
    n = t.shape[1] // tp
    return t[:, rank * n:(rank + 1) * n]


def shard_full_layer(cfg: ModelConfig, full: Dict[str, torch.Tensor], rank: int, tp: int):
    """Full (unsharded) HF-layout layer tensors -> this rank's fused shards."""
    d = cfg.head_dim
    q = full["q"].view(cfg.num_heads, d, -1)
    k = full["k"].view(cfg.num_kv_heads, d, -1)
    v = full["v"].view(cfg.num_kv_heads, d, -1)
    nq, _ = tp_heads(cfg, tp)
    k0, k1 = kv_head_range(cfg, tp, rank)
    qs = q[rank * nq:(rank + 1) * nq].reshape(-1, q.shape[-1])
    ks = k[k0:k1].reshape(-1, k.shape[-1])
    vs = v[k0:k1].reshape(-1, v.shape[-1])
    gate = _shard_rows(full["gate"], rank, tp)
    up = _shard_rows(full["up"], rank, tp)
    return {
        "wqkv": torch.cat([qs, ks, vs], 0).contiguous(),
        "wo": _shard_cols(full["o"], rank, tp).contiguous(),
        "wgu": torch.cat([gate, up], 0).contiguous(),
        "wd": _shard_cols(full["down"], rank, tp).contiguous(),
        "ln1": full["ln1"].contiguous(),
        "ln2": full["ln2"].contiguous(),
    }


def random_full_layer(cfg: ModelConfig, gen: torch.Generator, std: float, dtype):
    h, i, d = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim

    def rn(*shape):
        return (torch.randn(*shape, generator=gen, device=gen.device) * std).to(dtype)

    return {
        "q": rn(cfg.num_heads * d, h), "k": rn(cfg.num_kv_heads * d, h),
        "v": rn(cfg.num_kv_heads * d, h), "o": rn(h, cfg.num_heads * d),
        "gate": rn(i, h), "up": rn(i, h), "down": rn(h, i),
        "ln1": torch.ones(h, dtype=dtype), "ln2": torch.ones(h, dtype=dtype),
    }


def random_layer_fast(cfg: ModelConfig, rank: int, tp: int, layer: int, seed: int, std: float,
                      dtype, device) -> Dict[str, torch.Tensor]:
    """Per-shard random init generated directly on ``device`` (large models).

    Not TP-consistent (a TP=2 shard is not a slice of the TP=1 tensor) but
    statistically identical; used for benchmarking where the full unsharded
    tensors would be wasted work.
    """
    h, i, d = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    nq, nkv = tp_heads(cfg, tp)
    g = torch.Generator(device=device)
    g.manual_seed(seed * 1000003 + layer * 9176 + rank * 31 + 1)

    def rn(*shape):
        t = torch.empty(*shape, dtype=dtype, device=device)
        t.normal_(0.0, std, generator=g)
        return t

    return {
        "wqkv": rn((nq + 2 * nkv) * d, h), "wo": rn(h, nq * d),
        "wgu": rn(2 * (i // tp), h), "wd": rn(h, i // tp),
        "ln1": torch.ones(h, dtype=dtype, device=device),
        "ln2": torch.ones(h, dtype=dtype, device=device),
    }


# --------------------------------------------------------------------------------------
# safetensors checkpoints (HF Llama naming)
# --------------------------------------------------------------------------------------

class SafetensorsIndex:
    def __init__(self, ckpt_dir: str):
        from safetensors import safe_open  # noqa: F401

        self.dir = ckpt_dir
        idx = os.path.join(ckpt_dir, "model.safetensors.index.json")
        self.map: Dict[str, str] = {}
        if os.path.exists(idx):
            with open(idx) as f:
                self.map = {k: os.path.join(ckpt_dir, v) for k, v in json.load(f)["weight_map"].items()}
        else:
            from safetensors import safe_open

            for fn in sorted(glob.glob(os.path.join(ckpt_dir, "*.safetensors"))):
                with safe_open(fn, framework="pt") as f:
                    for k in f.keys():
                        self.map[k] = fn
        self._open: Dict[str, object] = {}

    def has(self, name: str) -> bool:
        return name in self.map

    def get(self, name: str) -> torch.Tensor:
        from safetensors import safe_open

        fn = self.map[name]
        if fn not in self._open:
            self._open[fn] = safe_open(fn, framework="pt")
        return self._open[fn].get_tensor(name)


def load_full_layer(idx: SafetensorsIndex, layer: int, dtype) -> Dict[str, torch.Tensor]:
    p = f"model.layers.{layer}."
    names = {
        "q": "self_attn.q_proj.weight", "k": "self_attn.k_proj.weight",
        "v": "self_attn.v_proj.weight", "o": "self_attn.o_proj.weight",
        "gate": "mlp.gate_proj.weight", "up": "mlp.up_proj.weight", "down": "mlp.down_proj.weight",
        "ln1": "input_layernorm.weight", "ln2": "post_attention_layernorm.weight",
    }
    return {k: idx.get(p + v).to(dtype) for k, v in names.items()}


# --------------------------------------------------------------------------------------
# AWQ (W4A16) checkpoints: AutoAWQ "GEMM" tensors per projection
# --------------------------------------------------------------------------------------
_HF_PROJ = {"q": "self_attn.q_proj", "k": "self_attn.k_proj", "v": "self_attn.v_proj",
            "o": "self_attn.o_proj", "gate": "mlp.gate_proj", "up": "mlp.up_proj",
            "down": "mlp.down_proj"}


def is_awq_checkpoint(idx: SafetensorsIndex) -> bool:
    cfg_path = os.path.join(idx.dir, "config.json")
    if os.path.exists(cfg_path):
        with open(cfg_path) as f:
            qc = json.load(f).get("quantization_config") or {}
        if str(qc.get("quant_method", "")).lower() == "awq":
            if int(qc.get("bits", 4)) != 4 or int(qc.get("group_size", 128)) != 128:
                raise ValueError("only 4-bit AWQ with group size 128 is supported")
            return True
    return idx.has("model.layers.0.self_attn.q_proj.qweight")


def load_awq_layer_shard(cfg: ModelConfig, idx: SafetensorsIndex, layer: int, rank: int, tp: int):
    """One layer of an AWQ checkpoint -> this rank's fused shards as (q, z, s)
    triples ([N, K] uint8, [N, K/128] uint8, [N, K/128] fp32).  The head / row /
    column slicing is the bf16 path's (:func:`shard_full_layer`) applied to q, z
    and s alike: groups run along K, so a row-parallel shard of K/tp columns
    (a multiple of 128) keeps whole groups."""
    from ..ops.quant import awq_unpack

    p = f"model.layers.{layer}."
    parts = {"q": {}, "z": {}, "s": {}}
    for name, hf in _HF_PROJ.items():
        q, z, s = awq_unpack(idx.get(p + hf + ".qweight"), idx.get(p + hf + ".qzeros"),
                             idx.get(p + hf + ".scales"))
        parts["q"][name], parts["z"][name], parts["s"][name] = q, z, s
    ln = {"ln1": idx.get(p + "input_layernorm.weight"),
          "ln2": idx.get(p + "post_attention_layernorm.weight")}
    sh = {k: shard_full_layer(cfg, dict(v, **ln), rank, tp) for k, v in parts.items()}
    out = {a: (sh["q"][a], sh["z"][a], sh["s"][a]) for a in ("wqkv", "wo", "wgu", "wd")}
    out.update(ln1=ln["ln1"], ln2=ln["ln2"])
    return out


def save_awq_checkpoint(cfg: ModelConfig, full_layers, embed, norm, lm_head, out_dir: str):
    """Quantize full-precision layers (RTN, group 128) and write them in the
    AutoAWQ GEMM layout with an HF ``quantization_config`` (tests and tooling)."""
    from safetensors.torch import save_file

    from ..ops.quant import awq_pack, quantize_w4

    save_hf_checkpoint(cfg, [], embed, norm, lm_head, out_dir)
    path = os.path.join(out_dir, "model.safetensors")
    from safetensors.torch import load_file

    t = load_file(path)
    for li, L in enumerate(full_layers):
        p = f"model.layers.{li}."
        for name, hf in _HF_PROJ.items():
            qw, qz, sc = awq_pack(*quantize_w4(L[name].to(torch.bfloat16)))
            t[p + hf + ".qweight"], t[p + hf + ".qzeros"], t[p + hf + ".scales"] = qw, qz, sc
        t[p + "input_layernorm.weight"] = L["ln1"].contiguous()
        t[p + "post_attention_layernorm.weight"] = L["ln2"].contiguous()
    save_file(t, path)
    with open(os.path.join(out_dir, "config.json")) as f:
        hf_cfg = json.load(f)
    hf_cfg["quantization_config"] = {"quant_method": "awq", "bits": 4, "group_size": 128,
                                     "zero_point": True, "version": "gemm"}
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(hf_cfg, f, indent=1)


def save_hf_checkpoint(cfg: ModelConfig, full_layers, embed, norm, lm_head: Optional[torch.Tensor],
                       out_dir: str):
    """Write an HF-layout safetensors checkpoint (used by tests and tooling)."""
    from safetensors.torch import save_file

    os.makedirs(out_dir, exist_ok=True)
    t = {"model.embed_tokens.weight": embed.contiguous(), "model.norm.weight": norm.contiguous()}
    if lm_head is not None and not cfg.tie_word_embeddings:
        t["lm_head.weight"] = lm_head.contiguous()
    inv = {"q": "self_attn.q_proj.weight", "k": "self_attn.k_proj.weight",
           "v": "self_attn.v_proj.weight", "o": "self_attn.o_proj.weight",
           "gate": "mlp.gate_proj.weight", "up": "mlp.up_proj.weight",
           "down": "mlp.down_proj.weight", "ln1": "input_layernorm.weight",
           "ln2": "post_attention_layernorm.weight"}
    for li, L in enumerate(full_layers):
        for k, v in L.items():
            t[f"model.layers.{li}.{inv[k]}"] = v.contiguous()
    save_file(t, os.path.join(out_dir, "model.safetensors"))
    hf = {
        "hidden_size": cfg.hidden_size, "num_hidden_layers": cfg.num_layers,
        "num_attention_heads": cfg.num_heads, "num_key_value_heads": cfg.num_kv_heads,
        "head_dim": cfg.head_dim, "intermediate_size": cfg.intermediate_size,
        "vocab_size": cfg.vocab_size, "rope_theta": cfg.rope_theta,
        "rope_scaling": cfg.rope_scaling, "rms_norm_eps": cfg.rms_norm_eps,
        "tie_word_embeddings": cfg.tie_word_embeddings,
        "max_position_embeddings": cfg.max_position_embeddings,
        "bos_token_id": cfg.bos_token_id, "eos_token_id": list(cfg.eos_token_ids),
        "architectures": ["LlamaForCausalLM"],
    }
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(hf, f, indent=1)
