"""Debug: GPU forward of tiny-2k with the packed decode GEMMs on/off."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fasttalk_llm_microservice_amd import ops
from fasttalk_llm_microservice_amd.models.config import MODELS
from fasttalk_llm_microservice_amd.models.llama import AttnMeta, LlamaModel
from fasttalk_llm_microservice_amd.ops import reference as ref

cfg = MODELS["tiny-2k"]
T = 40
def run(use_packed):
    m = LlamaModel(cfg, torch.device("cuda"), torch.bfloat16, max_model_len=512)
    m.use_packed = use_packed
    m.init_random(3)
    kv = m.allocate_kv_cache(8, 16)
    dev = "cuda"
    meta = AttnMeta(positions=torch.arange(T, dtype=torch.int32, device=dev),
                    slot_mapping=torch.arange(T, dtype=torch.int32, device=dev),
                    block_tables=torch.arange(8, dtype=torch.int32, device=dev)[None],
                    seq_lens=torch.tensor([T], dtype=torch.int32, device=dev),
                    logits_indices=torch.arange(T, device=dev),
                    q_start_loc=torch.tensor([0, T], dtype=torch.int32, device=dev),
                    tile_info=torch.tensor([[0, s] for s in range(0, T, 16)], dtype=torch.int32, device=dev).flatten(),
                    num_tiles=len(range(0, T, 16)))
    ids = torch.arange(100, 100 + T, dtype=torch.int32, device=dev)
    h = m.forward(ids, meta, kv)
    return m, h.float(), m.compute_logits(h).float()
m1, h1, l1 = run(True)
m0, h0, l0 = run(False)
print("packed layers:", m1.layers[0].wd_pk is not None, m1.lm_head_pk is not None, m0.ws is None)
print("hidden cos", torch.nn.functional.cosine_similarity(h1, h0, dim=-1).min().item())
print("logits cos", torch.nn.functional.cosine_similarity(l1, l0, dim=-1).min().item())
# pieces
L = m1.layers[0]
x = torch.randn(T, L.wd.shape[1], device="cuda").bfloat16()
ws = torch.empty(4 * T * L.wd.shape[0], device="cuda")
ops.skinny_gemm(x, L.wd_pk, ws=ws, splits=4, nt=4, u=-3)
y = ws.view(4, T, -1).sum(0)
print("down pk err", (y - x.float() @ L.wd.float().t()).abs().max().item())
res = torch.randn(T, cfg.hidden_size, device="cuda").bfloat16()
res2 = res.clone()
out = torch.empty(T, cfg.hidden_size, device="cuda").bfloat16()
ops.row_rmsnorm(out, L.ln1, 1e-5, T, ws=ws, splits=4, residual=res)
exp_res = (res2.float() + y)
print("row_rmsnorm residual err", (res.float() - exp_res).abs().max().item())
print("row_rmsnorm out err", (out.float() - ref.rmsnorm(exp_res.bfloat16(), L.ln1, 1e-5).float()).abs().max().item())
lg = ops.skinny_gemm(h0.bfloat16(), m1.lm_head_pk, splits=1, nt=2, u=-4).float()
print("lm_head pk err", (lg - h0.bfloat16().float() @ m1.lm_head.float().t()).abs().max().item())
