"""Sweep skinny_gemm (nt, u, splits) at decode shapes vs hipBLASLt; checks
numerics of every config against torch.  python bench/gemm_sweep.py [--m 50]"""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from fasttalk_llm_microservice_amd import ops
from kernel_bench import timeit  # noqa

ap = argparse.ArgumentParser()
ap.add_argument("--m", type=int, default=50)
ap.add_argument("--shapes", default="qkv:6144:4096,o:4096:4096,gate_up:28672:4096,down:4096:14336,lm_head:128256:4096")
a = ap.parse_args()
M = a.m
dev = "cuda"
torch.manual_seed(0)
best = {}
ws = torch.empty(32 * 64 * 128256, device=dev)
for spec in a.shapes.split(","):
    name, n, k = spec.split(":")
    n, k = int(n), int(k)
    W = (torch.randn(n, k, device=dev) * 0.02).bfloat16()
    x = torch.randn(M, k, device=dev).bfloat16()
    ref = F.linear(x, W).float()
    t_bl = timeit(lambda: F.linear(x, W), iters=100)
    print(f"{name} N={n} K={k}: hipblaslt {t_bl:.2f} us ({n*k*2/t_bl/1e3:.0f} GB/s)", flush=True)
    rows = []
    out = torch.empty(M, n, device=dev).bfloat16()
    for nt, u in ops.SKINNY_CONFIGS:
        for splits in (1, 2, 4, 8, 16, 32):
            if n % (16 * nt) or k % (64 * u * splits):
                continue
            blocks = (n // (64 * nt)) * splits
            if blocks < 64 or blocks > 8192:
                continue
            if splits == 1:
                fn = lambda: ops.skinny_gemm(x, W, out=out, nt=nt, u=u)
            else:
                fn = lambda: ops.skinny_gemm(x, W, ws=ws, splits=splits, nt=nt, u=u)
            fn()
            torch.cuda.synchronize()
            got = out.float() if splits == 1 else ws[: splits * M * n].view(splits, M, n).sum(0)
            err = (got - ref).abs().max().item()
            t = timeit(fn, iters=100)
            rows.append((t, nt, u, splits, blocks, err))
    rows.sort()
    for t, nt, u, splits, blocks, err in rows[:6]:
        print(f"   skinny nt={nt} u={u} splits={splits:2d} blocks={blocks:5d}: {t:7.2f} us ({n*k*2/t/1e3:5.0f} GB/s) err={err:.4f}", flush=True)
    bad = [r for r in rows if r[5] > 0.05]
    if bad:
        print("   !!! numerics failures:", bad[:3])
    best[name] = {"hipblaslt_us": t_bl, "best": rows[0][:5]}
print(json.dumps(best))
