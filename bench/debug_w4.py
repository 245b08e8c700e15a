"""Debug: GPU W4A16 model vs GPU bf16 model holding the dequantized weights vs the
CPU fp32 fake-quant model (same init), per-position logits cos / argmax agreement."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd.models.config import MODELS  # noqa: E402
from fasttalk_llm_microservice_amd.models.llama import AttnMeta, LlamaModel  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "tiny-2k"
T = int(sys.argv[2]) if len(sys.argv) > 2 else 40
cfg = MODELS[model]
g4 = LlamaModel(cfg, torch.device("cuda"), torch.bfloat16, max_model_len=512,
                quantization="w4").init_random(3, consistent=True)
c4 = LlamaModel(cfg, torch.device("cpu"), torch.float32, max_model_len=512,
                quantization="w4").init_random(3, consistent=True)
gb = LlamaModel(cfg, torch.device("cuda"), torch.bfloat16, max_model_len=512).init_random(
    3, consistent=True)
for Lg, Lc in zip(gb.layers, c4.layers):  # bf16 GPU model with the dequantized weights
    for a in ("wqkv", "wo", "wgu", "wd"):
        setattr(Lg, a, getattr(Lc, a).to("cuda", torch.bfloat16))
gb.use_packed = True
gb._prepare_packed()
cb = LlamaModel(cfg, torch.device("cpu"), torch.float32, max_model_len=512).init_random(
    3, consistent=True)
gbf = LlamaModel(cfg, torch.device("cuda"), torch.bfloat16, max_model_len=512).init_random(
    3, consistent=True)
bs, nblk = 16, 32
res = {}
for name, m in (("gpu_w4", g4), ("cpu_w4", c4), ("gpu_bf16_deq", gb), ("cpu_bf", cb),
                ("gpu_bf", gbf)):
    kv = m.allocate_kv_cache(nblk, bs)
    dev = m.device
    ids = torch.arange(100, 100 + T, dtype=torch.int32, device=dev)
    meta = AttnMeta(
        positions=torch.arange(T, dtype=torch.int32, device=dev),
        slot_mapping=torch.arange(T, dtype=torch.int32, device=dev),
        block_tables=torch.arange(nblk, dtype=torch.int32, device=dev)[None],
        seq_lens=torch.tensor([T], dtype=torch.int32, device=dev),
        logits_indices=torch.arange(T, device=dev),
        q_start_loc=torch.tensor([0, T], dtype=torch.int32, device=dev if dev.type == "cuda" else "cpu"),
        tile_info=torch.tensor([[0, s] for s in range(0, T, 16)], dtype=torch.int32,
                               device=dev).flatten(),
        num_tiles=len(range(0, T, 16)))
    h = m.forward(ids, meta, kv)
    res[name] = m.compute_logits(h).float().cpu()


def cmp(a, b):
    cos = torch.nn.functional.cosine_similarity(res[a], res[b], dim=-1)
    agree = (res[a].argmax(-1) == res[b].argmax(-1)).float().mean().item()
    print(f"{a:>13} vs {b:<13} cos min {cos.min().item():.5f} mean {cos.mean().item():.5f} "
          f"argmax agree {agree:.3f}")


cmp("gpu_w4", "cpu_w4")
cmp("gpu_w4", "gpu_bf16_deq")
cmp("gpu_bf16_deq", "cpu_w4")
cmp("gpu_bf", "cpu_bf")

from fasttalk_llm_microservice_amd.ops import quant as Q  # noqa: E402

for a, proj in (("wqkv", "qkv"), ("wo", "o"), ("wgu", "gu"), ("wd", "down")):
    qq = g4.layers[0].q4[proj]
    W = Q.W4Weight(qq.wq.cpu(), qq.sz.cpu(), qq.n, qq.k)
    dq = Q.dequantize_w4(*Q.unpack_w4(W))
    ref_w = getattr(c4.layers[0], a)
    d = (dq - ref_w).abs()
    print(f"{proj}: max |gpu deq - cpu deq| {d.max().item():.3e}, mismatches {(d > 1e-6).sum().item()}"
          f" of {d.numel()}")
    # kernel on this exact weight vs fp32 matmul
    x = torch.randn(40, qq.k, device="cuda").bfloat16()
    y = Q.w4_gemm(x, qq).float().cpu()
    r = x.float().cpu() @ dq.t()
    print(f"   kernel vs fp32 on same weight: rel max err {((y - r).abs().max() / r.abs().max()).item():.2e}")
