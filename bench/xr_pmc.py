"""Runs one decode GEMM config repeatedly (for rocprofv3 --pmc passes):
python bench/xr_pmc.py [--proj gu] [--m 50]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096, (1, -5, 2)), "o": (4096, 4096, (1, -5, 4)),
          "gu": (28672, 4096, (2, -6, 1)), "down": (4096, 14336, (1, -5, 4))}
ap = argparse.ArgumentParser()
ap.add_argument("--proj", default="gu")
ap.add_argument("--m", type=int, default=50)
a = ap.parse_args()
n, k, (nt, u, sp) = SHAPES[a.proj]
ws = torch.empty(8 * 64 * 28672, device="cuda")
Ws = [ops.pack_weight((torch.randn(n, k, device="cuda") * 0.02).bfloat16()) for _ in range(4)]
x = torch.randn(a.m, k, device="cuda").bfloat16()
for i in range(64):
    ops.skinny_gemm(x, Ws[i % 4], ws=ws if sp > 1 else None, splits=sp, nt=nt, u=u)
torch.cuda.synchronize()
print("done")
