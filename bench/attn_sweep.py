"""Decode-attention sweep: us/call and effective KV bandwidth of the paged MFMA
decode kernel (csrc/kernels/attn_decode.hip) at Llama-3-8B head shapes over
(batch, context).  Lengths are ragged (uniform in [ctx/2, ctx], first = ctx)
unless --uniform; KV blocks are scattered (random permutation), like a pool
that has served many sessions.

python bench/attn_sweep.py [--nq 32 --nkv 8] [--uniform]
FT_DECODE_RING=2|3|4 selects the kernel's register-ring depth (default 2);
FT_DECODE_MIN_TILES the partition's minimum 16-token tiles per wave (default 8);
FT_DECODE_WPC workgroups per CU (1-3, default 1); FT_DECODE_WAVES waves per workgroup (1 / 2 / 4,
default 2).
--fused: the in-launch combine the engine uses (decode tickets) instead of the
separate combine kernel.  --shapes "1:512,1:3000" overrides the shape list.
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

SHAPES = [(1, 512), (1, 8192), (8, 2048), (50, 640), (50, 3000), (50, 4500), (64, 1024),
          (64, 4096), (256, 1024)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, default=32)
    ap.add_argument("--nkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--uniform", action="store_true")
    ap.add_argument("--fused", action="store_true")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--bs", type=int, default=16, help="KV block size (tokens)")
    a = ap.parse_args()
    shapes = [tuple(int(v) for v in x.split(":")) for x in a.shapes.split(",")] if a.shapes else SHAPES
    nq, nkv, d, bs = a.nq, a.nkv, a.d, a.bs
    dev = "cuda"
    for B, ctx in shapes:
        nblk = math.ceil(ctx / bs)
        nblocks = B * nblk + 8
        kc = torch.randn(nblocks, nkv, bs, d, device=dev).bfloat16()
        vc = torch.randn(nblocks, nkv, d, bs, device=dev).bfloat16()
        bt = torch.randperm(nblocks, device=dev)[: B * nblk].int().view(B, nblk)
        if a.uniform:
            sl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        else:
            sl = torch.randint(max(1, ctx // 2), ctx + 1, (B,), dtype=torch.int32, device=dev)
            sl[0] = ctx
        q = torch.randn(B, (nq + 2 * nkv) * d, device=dev).bfloat16()
        out = torch.empty(B, nq * d, device=dev).bfloat16()
        n_out, n_ml = ops.decode_workspace(B, nq, nkv, d)
        tmp_o = torch.empty(n_out, device=dev)
        tmp_ml = torch.empty(n_ml, device=dev)
        nbytes = int(sl.sum().item()) * nkv * d * 2 * 2
        cnt = ops.decode_counters(B, nkv, dev) if a.fused else None
        us = timeit(lambda: ops.decode_attention(out, q, kc, vc, bt, sl, tmp_o, tmp_ml, nq, nkv, d,
                                                 d ** -0.5, counters=cnt), iters=100, warmup=10)
        print(json.dumps({"B": B, "ctx": ctx, "uniform": a.uniform, "bs": bs,
                          "ring": int(os.environ.get("FT_DECODE_RING", "2")),
                          "min_tiles": int(os.environ.get("FT_DECODE_MIN_TILES", "8")),
                          "wpc": int(os.environ.get("FT_DECODE_WPC", "1")),
                          "fused": a.fused,
                          "us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)}), flush=True)
        del kc, vc


if __name__ == "__main__":
    main()
