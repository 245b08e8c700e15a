import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
os.environ["FT_W4_PREFILL_IMAGE"] = "0"
from fasttalk_llm_microservice_amd import ops
from fasttalk_llm_microservice_amd.ops import quant as Q
from fasttalk_llm_microservice_amd.models.llama import LlamaModel
from fasttalk_llm_microservice_amd.models.config import MODELS
g = LlamaModel(MODELS["tiny-2k"], torch.device("cuda"), torch.bfloat16, max_model_len=512, quantization="w4").init_random(3, consistent=True)
L = g.layers[0]
for p in ("qkv", "o", "gu", "down"):
    q = L.q4[p]
    a = g._w4_packed(q).clone()
    b = ops.pack_weight(Q.w4_dequant(q))
    print(p, q.n, q.k, torch.equal(a, b), (a.float() - b.float()).abs().max().item())
