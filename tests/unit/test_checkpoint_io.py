"""Weights and tokenizer I/O (E14 / E3): an HF-layout safetensors checkpoint
written from random weights loads back into the engine (config.json ->
ModelConfig, q/k/v and gate/up fused and TP-sharded) and reproduces the
in-memory model's greedy tokens; a tokenizer.json on disk loads through the
same path a real Llama-3 tokenizer would; the weights are read with
safetensors only (no pickle)."""
import json
import os

import numpy as np
import torch

from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
from fasttalk_llm_microservice_amd.engine.tokenizer import Tokenizer, get_tokenizer
from fasttalk_llm_microservice_amd.models import weights as W
from fasttalk_llm_microservice_amd.models.config import MODELS, resolve_model


def _write_ckpt(cfg, out_dir, seed=5):
    g = torch.Generator().manual_seed(seed)
    layers = [W.random_full_layer(cfg, g, 0.02, torch.float32) for _ in range(cfg.num_layers)]
    embed = torch.randn(cfg.vocab_size, cfg.hidden_size, generator=g) * 0.02
    norm = torch.ones(cfg.hidden_size) + 0.05 * torch.randn(cfg.hidden_size, generator=g)
    lm_head = torch.randn(cfg.vocab_size, cfg.hidden_size, generator=g) * 0.02
    W.save_hf_checkpoint(cfg, layers, embed, norm, lm_head, out_dir)
    return layers, embed, norm, lm_head


def test_checkpoint_roundtrip_matches_in_memory_model(tmp_path):
    cfg = MODELS["tiny"]
    ckpt = str(tmp_path / "tiny-ckpt")
    layers, embed, norm, lm_head = _write_ckpt(cfg, ckpt)
    loaded_cfg = resolve_model(ckpt)
    assert (loaded_cfg.hidden_size, loaded_cfg.num_layers, loaded_cfg.num_kv_heads) == \
        (cfg.hidden_size, cfg.num_layers, cfg.num_kv_heads)
    eng = LLMEngine(EngineConfig(model="tiny", weights=ckpt, device="cpu", num_kv_blocks=128,
                                 max_model_len=512))
    m = eng.runner.model
    # fused/sharded layout of layer 0 equals the checkpoint tensors
    L0 = layers[0]
    torch.testing.assert_close(m.layers[0].wqkv, torch.cat([L0["q"], L0["k"], L0["v"]], 0))
    torch.testing.assert_close(m.layers[0].wgu, torch.cat([L0["gate"], L0["up"]], 0))
    torch.testing.assert_close(m.norm, norm)
    torch.testing.assert_close(m.lm_head, lm_head)
    # the engine generates deterministically from the loaded weights, and a
    # second load gives the same tokens
    sp = SamplingParams(temperature=0, max_tokens=6, ignore_eos=True)
    a = eng.generate([[1, 2, 3, 4]], sp)
    b = LLMEngine(EngineConfig(model="tiny", weights=ckpt, device="cpu", num_kv_blocks=128,
                               max_model_len=512)).generate([[1, 2, 3, 4]], sp)
    assert a == b and len(a[0]) == 6


def test_checkpoint_tp_shards_cover_full_tensors(tmp_path):
    cfg = MODELS["tiny-gqa4"]
    full = W.random_full_layer(cfg, torch.Generator().manual_seed(1), 0.02, torch.float32)
    shards = [W.shard_full_layer(cfg, full, r, 2) for r in range(2)]
    # row-parallel O / down: concatenating the column shards restores the full weight
    torch.testing.assert_close(torch.cat([s["wo"] for s in shards], 1), full["o"])
    torch.testing.assert_close(torch.cat([s["wd"] for s in shards], 1), full["down"])
    nq, nkv = W.tp_heads(cfg, 2)
    assert shards[0]["wqkv"].shape[0] == (nq + 2 * nkv) * cfg.head_dim


def test_tokenizer_json_on_disk(tmp_path):
    syn = get_tokenizer()
    path = tmp_path / "tokenizer.json"
    syn.hf.save(str(path))
    tok = Tokenizer(str(tmp_path))  # a checkpoint dir with tokenizer.json
    text = "Hello there — how's it going? 123"
    assert tok.encode(text) == syn.encode(text)
    assert tok.eot_id == 128009 and tok.bos_id == 128000
    assert tok.decode(tok.encode(text)) == text
    with open(path) as f:
        assert "<|eot_id|>" in json.dumps(json.load(f)["added_tokens"])
