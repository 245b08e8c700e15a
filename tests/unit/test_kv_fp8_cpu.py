"""fp8 (e4m3) KV cache on the CPU backend: config parsing, the reference write /
read paths the GPU kernels are checked against (tests/test_kv_fp8_gpu.py), and an
engine serving from fp8 caches end to end (prefix reuse, host swap)."""
import numpy as np
import pytest
import torch

from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
from fasttalk_llm_microservice_amd.ops import reference as ref

F8 = torch.float8_e4m3fn


def test_config_kv_cache_dtype(monkeypatch):
    assert EngineConfig(device="cpu").kv_torch_dtype(torch.bfloat16) == torch.bfloat16
    assert EngineConfig(device="cpu", kv_cache_dtype="fp8").kv_torch_dtype(torch.bfloat16) == F8
    monkeypatch.setenv("ENGINE_KV_CACHE_DTYPE", "fp8")
    assert EngineConfig.from_env().kv_torch_dtype(torch.float32) == F8
    with pytest.raises(ValueError):
        EngineConfig(kv_cache_dtype="int3").kv_torch_dtype(torch.bfloat16)


def test_reference_write_clamps_and_reads_back():
    nq, nkv, d, bs = 4, 2, 64, 16
    t = 5
    qkv = torch.randn(t, (nq + 2 * nkv) * d) * 4
    qkv[0, (nq + nkv) * d] = 1e4          # past e4m3's range: clamped, not NaN
    cs = ref.rope_cos_sin(d, 64, 500000.0, None, "cpu")
    pos = torch.arange(t, dtype=torch.int32)
    slots = torch.arange(t, dtype=torch.int32)
    k8 = torch.zeros(2, nkv, bs, d, dtype=F8)
    v8 = torch.zeros(2, nkv, d, bs, dtype=F8)
    kf = torch.zeros(2, nkv, bs, d)
    vf = torch.zeros(2, nkv, d, bs)
    ref.rope_kv_write(qkv.clone(), pos, cs, slots, k8, v8, nq, nkv, d)
    ref.rope_kv_write(qkv.clone(), pos, cs, slots, kf, vf, nq, nkv, d)
    assert torch.isfinite(k8.float()).all() and torch.isfinite(v8.float()).all()
    assert v8[0, 0, 0, 0].float().item() == 448.0
    # every stored value is the nearest e4m3 of the fp32 one (within half a step: 1/16)
    err = (v8.float() - vf.clamp(-448, 448)).abs()
    assert (err <= vf.abs().clamp(-448, 448) / 16 + 2 ** -10).all()
    # attention over the fp8 cache == attention over its dequantized values
    q = torch.randn(t, nq, d)
    bt = torch.tensor([[0, 1]], dtype=torch.int32)
    sl = torch.tensor([t], dtype=torch.int32)
    qsl = torch.tensor([0, t], dtype=torch.int32)
    a = ref.paged_attention(q, k8, v8, bt, sl, qsl, d ** -0.5)
    b = ref.paged_attention(q, k8.float(), v8.float(), bt, sl, qsl, d ** -0.5)
    assert torch.equal(a, b)


def _prompts(n, lens, seed=0):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 120000, l).tolist() for l in lens[:n]]


def test_cpu_engine_serves_from_fp8_cache():
    prompts = _prompts(4, [7, 20, 33, 50])
    sp = SamplingParams(temperature=0.0, max_tokens=12, ignore_eos=True)
    e = LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=64, max_model_len=512,
                               max_num_seqs=8, kv_cache_dtype="fp8", swap_space_gb=0.01))
    r = e.runner
    assert r.kv[0][0].dtype == F8 and r.kv[0][1].dtype == F8
    out = e.generate(prompts, sp)
    assert all(len(o) == 12 for o in out)
    assert e.generate(prompts[:2], sp) == out[:2]        # prefix-cache hits on fp8 blocks
    # host swap moves fp8 bytes both ways
    for k, v in r.kv:
        k.copy_(torch.randn(k.shape).to(F8))
        v.copy_(torch.randn(v.shape).to(F8))
    before = [(k[[3, 7]].view(torch.uint8).clone(), v[[3, 7]].view(torch.uint8).clone()) for k, v in r.kv]
    r.swap([(3, 0), (7, 1)], [])
    r.swap([], [(0, 10), (1, 11)])
    for (k, v), (k0, v0) in zip(r.kv, before):
        assert torch.equal(k[[10, 11]].view(torch.uint8), k0) and torch.equal(v[[10, 11]].view(torch.uint8), v0)


def test_fp8_pool_holds_twice_the_tokens():
    def per_block(kv):
        e = LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=32, max_model_len=256,
                                   max_num_seqs=4, kv_cache_dtype=kv))
        k, v = e.runner.kv[0]
        return k.numel() * k.element_size() + v.numel() * v.element_size()

    # the CPU backend computes in fp32: fp8 blocks are a quarter of its bytes (half of bf16's)
    assert per_block("fp8") * 4 == per_block("auto")
