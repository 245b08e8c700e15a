"""W4A16 / AWQ (E9, K14): the quantizer, the kernel's packed image, the AutoAWQ
checkpoint layout and the engine's quantized CPU path.  The packed image is
checked against an element-by-element emulation of what ``w4a16.hip`` computes
from it (lane / word / nibble decoding), so a layout bug shows up on the CPU.
No real AWQ checkpoint is available offline: the AutoAWQ layout is pinned by
the round trip through :func:`awq_pack` only (parity with a downloaded
checkpoint is unpinned)."""
import numpy as np
import pytest
import torch

from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
from fasttalk_llm_microservice_amd.models import weights as W
from fasttalk_llm_microservice_amd.models.config import MODELS
from fasttalk_llm_microservice_amd.ops import quant as Q


def _w(n, k, seed=0):
    return torch.randn(n, k, generator=torch.Generator().manual_seed(seed)) * 0.05


def test_quantize_error_bound_and_range():
    w = _w(64, 512)
    q, z, s = Q.quantize_w4(w)
    assert q.max() <= 15 and z.max() <= 15
    err = (Q.dequantize_w4(q, z, s) - w).abs().view(64, 4, 128).amax(-1)
    assert (err <= s * 1.0001).all()


def test_packed_image_matches_kernel_semantics():
    n, k = 32, 256
    q, z, s = Q.quantize_w4(_w(n, k, 1))
    packed = Q.pack_w4(q, z, s)
    wq = packed.wq.numpy().view(np.uint32).reshape(n // 16, k // 128, 64, 4)
    sz = packed.sz.numpy().reshape(n // 16, k // 128, 16, 2)
    emu = np.zeros((n, k))
    for t in range(n // 16):
        for gr in range(k // 128):
            for lane in range(64):
                r, g = lane & 15, lane >> 4
                sc, zz = sz[t, gr, r]
                for h in range(4):
                    word = int(wq[t, gr, lane, h])
                    kb = 128 * gr + 64 * (h >> 1) + 16 * g + 8 * (h & 1)
                    for i in range(4):  # bf16 pair i = (nibble i, nibble i + 4)
                        emu[16 * t + r, kb + 2 * i] = ((word >> (4 * i)) & 15) + 128 - zz
                        emu[16 * t + r, kb + 2 * i + 1] = ((word >> (4 * i + 16)) & 15) + 128 - zz
                        emu[16 * t + r, kb + 2 * i:kb + 2 * i + 2] *= sc
    np.testing.assert_allclose(emu, Q.dequantize_w4(q, z, s).numpy(), rtol=0, atol=1e-7)
    q2, z2, s2 = Q.unpack_w4(packed)
    assert torch.equal(q2, q) and torch.equal(z2, z) and torch.allclose(s2, s)


def test_awq_layout_round_trip():
    q, z, s = Q.quantize_w4(_w(48, 384, 2))
    qw, qz, sc = Q.awq_pack(q, z, s)
    assert qw.shape == (384, 6) and qz.shape == (3, 6) and sc.shape == (3, 48)
    assert qw.dtype == torch.int32 and sc.dtype == torch.float16
    q2, z2, s2 = Q.awq_unpack(qw, qz, sc)
    assert torch.equal(q2, q) and torch.equal(z2, z)
    torch.testing.assert_close(s2, s, rtol=1e-3, atol=0)
    # nibble i of word c holds column 8c + AWQ_ORDER[i]
    assert (qw[0, 0].item() >> 4) & 15 == q[Q.AWQ_ORDER[1], 0].item()


def test_w4_cpu_gemm_is_dequant_matmul():
    q, z, s = Q.quantize_w4(_w(64, 256, 3))
    packed = Q.pack_w4(q, z, s)
    x = torch.randn(5, 256)
    torch.testing.assert_close(Q.w4_gemm(x, packed), x @ Q.dequantize_w4(q, z, s).t())


def _full_layers(cfg, seed):
    g = torch.Generator().manual_seed(seed)
    return [W.random_full_layer(cfg, g, 0.02, torch.float32) for _ in range(cfg.num_layers)]


def test_awq_checkpoint_loads_and_matches_rtn_engine(tmp_path):
    cfg = MODELS["tiny"]
    layers = _full_layers(cfg, 4)
    g = torch.Generator().manual_seed(9)
    embed = torch.randn(cfg.vocab_size, cfg.hidden_size, generator=g) * 0.02
    norm = torch.ones(cfg.hidden_size)
    lm = torch.randn(cfg.vocab_size, cfg.hidden_size, generator=g) * 0.02
    awq_dir, bf_dir = str(tmp_path / "awq"), str(tmp_path / "bf")
    W.save_awq_checkpoint(cfg, layers, embed, norm, lm, awq_dir)
    W.save_hf_checkpoint(cfg, layers, embed, norm, lm, bf_dir)
    base = dict(model="tiny", device="cpu", num_kv_blocks=128, max_model_len=512)
    awq = LLMEngine(EngineConfig(weights=awq_dir, **base))
    rtn = LLMEngine(EngineConfig(weights=bf_dir, quantization="w4", **base))
    assert awq.runner.model.quant == "awq"
    m = awq.runner.model
    L0 = layers[0]
    deq = {k: Q.dequantize_w4(*Q.quantize_w4(L0[k].bfloat16()))
           for k in ("q", "k", "v", "gate", "up")}
    torch.testing.assert_close(m.layers[0].wqkv, torch.cat([deq["q"], deq["k"], deq["v"]], 0),
                               rtol=1e-3, atol=1e-5)  # scales go through fp16 in the AWQ file
    torch.testing.assert_close(m.layers[0].wgu, torch.cat([deq["gate"], deq["up"]], 0),
                               rtol=1e-3, atol=1e-5)
    sp = SamplingParams(temperature=0, max_tokens=8, ignore_eos=True)
    assert awq.generate([[5, 6, 7, 8]], sp) == rtn.generate([[5, 6, 7, 8]], sp)


@pytest.mark.parametrize("tp", [2])
def test_awq_tp_shards_concatenate_to_full(tmp_path, tp):
    cfg = MODELS["tiny-2k"]
    layers = _full_layers(cfg, 6)[:1]
    c = cfg.__class__(**{**cfg.__dict__, "num_layers": 1})
    d = str(tmp_path / "awq")
    W.save_awq_checkpoint(c, layers, torch.zeros(c.vocab_size, c.hidden_size),
                          torch.ones(c.hidden_size), None, d)
    idx = W.SafetensorsIndex(d)
    full = W.load_awq_layer_shard(c, idx, 0, 0, 1)
    shards = [W.load_awq_layer_shard(c, idx, 0, r, tp) for r in range(tp)]
    for a in ("wo", "wd"):  # row parallel: K (and the groups) split
        for i in range(3):
            assert torch.equal(torch.cat([s[a][i] for s in shards], 1), full[a][i])
    # column parallel gate|up: each rank holds its slice of gate and of up
    n_i = c.intermediate_size
    gate = torch.cat([s["wgu"][0][:n_i // tp] for s in shards], 0)
    assert torch.equal(gate, full["wgu"][0][:n_i])
