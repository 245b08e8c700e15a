"""Runs one packed_gemm config (or hipBLASLt) back to back, for rocprofv3 --pmc.
python bench/pg_pmc.py --m 4096 --n 28672 --k 4096 --cfg 0 [--blas]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=4096)
ap.add_argument("--n", type=int, default=28672)
ap.add_argument("--k", type=int, default=4096)
ap.add_argument("--cfg", type=int, default=0)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--blas", action="store_true")
a = ap.parse_args()
w = torch.randn(a.n, a.k, device="cuda").bfloat16() * 0.02
x = torch.randn(a.m, a.k, device="cuda").bfloat16()
wp = ops.pack_weight(w)
out = torch.empty(a.m, a.n, device="cuda").bfloat16()
for _ in range(a.iters):
    if a.blas:
        F.linear(x, w)
    else:
        ops.packed_gemm(x, wp, out=out, cfg=a.cfg)
torch.cuda.synchronize()
print("done")
