"""Per-kernel micro-benchmarks at Llama-3-8B decode / prefill shapes.

Times each HIP kernel (and the hipBLASLt GEMMs it sits between) with HIP
events over many back-to-back launches and reports us/call and the effective
HBM bandwidth of the bytes the op must move.

python bench/kernel_bench.py [--batch 50] [--ctx 640]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402


def timeit(fn, iters=200, warmup=20):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=50)
    ap.add_argument("--ctx", type=int, default=640)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = "cuda"
    B, ctx = a.batch, a.ctx
    H, I, nq, nkv, d, V = 4096, 14336, 32, 8, 128, 128256
    bs = 16
    res = {}

    def rep(name, us, nbytes):
        res[name] = {"us": round(us, 2), "GBps": round(nbytes / us / 1e3, 1)}
        print(f"{name:34s} {us:9.2f} us  {nbytes / us / 1e3:8.1f} GB/s", flush=True)

    torch.manual_seed(0)
    x = torch.randn(B, H, device=dev).bfloat16()
    r = torch.randn(B, H, device=dev).bfloat16()
    w = torch.ones(H, device=dev).bfloat16()
    if not a.only or "norm" in a.only:
        rep("fused_add_rmsnorm", timeit(lambda: ops.fused_add_rmsnorm(x, r, w, 1e-5)), B * H * 2 * 4)
    gu = torch.randn(B, 2 * I, device=dev).bfloat16()
    if not a.only or "silu" in a.only:
        rep("silu_mul", timeit(lambda: ops.silu_mul(gu)), B * I * 2 * 3)
    # GEMMs (hipBLASLt via torch)
    for name, n, k in [("qkv", (nq + 2 * nkv) * d, H), ("o", H, nq * d), ("gate_up", 2 * I, H),
                       ("down", H, I), ("lm_head", V, H)]:
        if a.only and name not in a.only and "gemm" not in a.only:
            continue
        W = torch.randn(n, k, device=dev).bfloat16() * 0.02
        xx = torch.randn(B, k, device=dev).bfloat16()
        rep(f"hipblaslt {name} [{B}x{k}]x[{k}x{n}]", timeit(lambda: F.linear(xx, W)), n * k * 2)
        if B <= 64 and n % 64 == 0 and k % 64 == 0:
            out = torch.empty(B, n, device=dev).bfloat16()
            Wp = ops.pack_weight(W)
            rep(f"packed   {name}", timeit(lambda: ops.skinny_gemm(xx, Wp, out=out, nt=2, u=-3)),
                n * k * 2)
            ref = F.linear(xx, W).float()
            err = (out.float() - ref).abs().max().item()
            print(f"   max err vs hipblaslt {err:.4f}")
    # attention
    nblk_per = math.ceil(ctx / bs)
    nblocks = B * nblk_per + 8
    kc = torch.randn(nblocks, nkv, bs, d, device=dev).bfloat16()
    vc = torch.randn(nblocks, nkv, d, bs, device=dev).bfloat16()   # transposed V blocks
    bt = torch.randperm(nblocks, device=dev)[: B * nblk_per].int().view(B, nblk_per)
    sl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
    q = torch.randn(B, (nq + 2 * nkv) * d, device=dev).bfloat16()
    out = torch.empty(B, nq * d, device=dev).bfloat16()
    n_out, n_ml = ops.decode_workspace(B, nq, nkv, d)
    tmp_o = torch.empty(n_out, device=dev)
    tmp_ml = torch.empty(n_ml, device=dev)
    if not a.only or "attn" in a.only:
        rep(f"decode_attn B={B} ctx={ctx}",
            timeit(lambda: ops.decode_attention(out, q, kc, vc, bt, sl, tmp_o, tmp_ml, nq, nkv, d,
                                                d ** -0.5)), B * ctx * nkv * d * 2 * 2)
    slots = torch.arange(B, dtype=torch.int32, device=dev)
    pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=dev)
    cs = ops.reference.rope_cos_sin(d, 8192, 500000.0, None, dev)
    if not a.only or "rope" in a.only:
        rep("rope_kv_write", timeit(lambda: ops.rope_kv_write(q, pos, cs, slots, kc, vc, nq, nkv, d)),
            B * (nq + 2 * nkv) * d * 2 * 2)
    logits = torch.randn(B, V, device=dev).bfloat16()
    temp = torch.full((B,), 0.7, device=dev)
    tp = torch.full((B,), 0.9, device=dev)
    tk0 = torch.zeros(B, dtype=torch.int32, device=dev)
    tk40 = torch.full((B,), 40, dtype=torch.int32, device=dev)
    seeds = torch.arange(B, dtype=torch.int64, device=dev)
    steps = torch.zeros(B, dtype=torch.int32, device=dev)
    if not a.only or "sample" in a.only:
        rep("sample greedy", timeit(lambda: ops.sample(logits, temp * 0, tp, tk0, seeds, steps)), B * V * 2)
        rep("sample T=0.7 top_p=0.9", timeit(lambda: ops.sample(logits, temp, tp, tk0, seeds, steps)), B * V * 2)
        rep("sample T=0.7 top_k=40 top_p=0.9", timeit(lambda: ops.sample(logits, temp, tp, tk40, seeds, steps)), B * V * 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
