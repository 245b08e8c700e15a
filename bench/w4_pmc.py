"""Runs one W4A16 decode GEMM config repeatedly (for rocprofv3 --pmc passes):
python bench/w4_pmc.py [--proj gu] [--m 50]   (the engine's W4_PLAN entry at 64 rows)"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd.models.llama import w4_cfg  # noqa: E402
from fasttalk_llm_microservice_amd.ops import quant as Q  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (28672, 4096), "down": (4096, 14336)}
ap = argparse.ArgumentParser()
ap.add_argument("--proj", default="gu")
ap.add_argument("--m", type=int, default=50)
ap.add_argument("--cfg", default="", help="nt,splits,xr override of the plan entry")
a = ap.parse_args()
n, k = SHAPES[a.proj]
nt, sp, xr = w4_cfg(a.proj, a.m)
if a.cfg:
    nt, sp, xr = (int(v) for v in a.cfg.split(","))
silu = a.proj == "gu"
ws = torch.empty(16 * 64 * 28672, device="cuda")
Ws = []
for _ in range(4):
    q, z, s = Q.quantize_w4(torch.randn(n, k, device="cuda") * 0.02)
    Ws.append(Q.pack_w4(q, z, s))   # (the SiLU epilogue's column pairing is layout-only)
x = torch.randn(a.m, k, device="cuda").bfloat16()
out = torch.empty(a.m, n, device="cuda").bfloat16()   # silu writes n / 2 of it
for i in range(64):
    if sp > 1:
        Q.w4_gemm(x, Ws[i % 4], ws=ws, splits=sp, nt=nt, xr=xr)
    else:
        Q.w4_gemm(x, Ws[i % 4], out=out, nt=nt, xr=xr, silu=silu and bool(xr))
torch.cuda.synchronize()
print("done", a.proj, (nt, sp, xr))
