"""Decode-attention split sweep: us/call and effective KV bandwidth of the paged
decode kernel at Llama-3-8B head shapes over (batch, context, splits).

python bench/attn_sweep.py [--nq 32 --nkv 8]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402
from kernel_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, default=32)
    ap.add_argument("--nkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    a = ap.parse_args()
    nq, nkv, d, bs = a.nq, a.nkv, a.d, 16
    dev = "cuda"
    res = []
    for B, ctx in [(1, 512), (1, 8192), (8, 2048), (50, 640), (64, 1024), (64, 4096), (256, 1024)]:
        nblk = math.ceil(ctx / bs)
        nblocks = B * nblk + 8
        kc = torch.randn(nblocks, nkv, bs, d, device=dev).bfloat16()
        vc = torch.randn(nblocks, nkv, bs, d, device=dev).bfloat16()
        bt = torch.randperm(nblocks, device=dev)[: B * nblk].int().view(B, nblk)
        sl = torch.randint(max(1, ctx // 2), ctx + 1, (B,), dtype=torch.int32, device=dev)
        sl[0] = ctx
        q = torch.randn(B, (nq + 2 * nkv) * d, device=dev).bfloat16()
        out = torch.empty(B, nq * d, device=dev).bfloat16()
        tmp_o = torch.empty(B * nq * 64 * d, device=dev)
        tmp_ml = torch.empty(B * nq * 64 * 2, device=dev)
        nbytes = int(sl.sum().item()) * nkv * d * 2 * 2
        row = {"B": B, "ctx": ctx, "policy": ops.decode_splits(B, nkv)}
        for s in (1, 2, 4, 8, 16, 32, 64):
            us = timeit(lambda: ops.decode_attention(out, q, kc, vc, bt, sl, tmp_o, tmp_ml, nq, nkv, d,
                                                     s, d ** -0.5), iters=100, warmup=10)
            row[f"s{s}"] = round(us, 2)
        best = min((row[f"s{s}"], s) for s in (1, 2, 4, 8, 16, 32, 64))
        row["best"] = best[1]
        row["best_GBps"] = round(nbytes / best[0] / 1e3, 1)
        row["policy_GBps"] = round(nbytes / row[f"s{row['policy']}"] / 1e3, 1)
        print(json.dumps(row), flush=True)
        res.append(row)
        del kc, vc


if __name__ == "__main__":
    main()
