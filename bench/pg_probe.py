"""Packed-image GEMMs vs hipBLASLt on row-major weights at Llama-3-8B
projection shapes above the decode row counts: the "xc" streaming kernel
(skinny_gemm.hip, <= 128 rows, split-K slabs) and packed_gemm.hip (any M, tile
configs, split-K slabs) -- correctness against F.linear and time (us, TF/s).
Slab variants are timed together with a slab_store pass (the reduction the
epilogue kernels otherwise fold in), so the numbers are conservative.

python bench/pg_probe.py [--rows 80,128,256,512,1024,4096] [--only qkv,gu]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (28672, 4096), "down": (4096, 14336),
          "lm": (128256, 4096)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="80,128,256,512,1024,4096")
    ap.add_argument("--only", default="")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cfgs", default="0,1,2,3,4,5,6")
    ap.add_argument("--splits", default="1,2,4,8,16")
    a = ap.parse_args()
    torch.manual_seed(0)
    for name, (n, k) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        w = torch.randn(n, k, device="cuda").bfloat16() * 0.02
        wp = ops.pack_weight(w)
        ws = torch.empty(64 << 20, device="cuda")
        for m in [int(v) for v in a.rows.split(",")]:
            x = torch.randn(m, k, device="cuda").bfloat16()
            ref = F.linear(x, w).float()
            out = torch.empty(m, n, device="cuda").bfloat16()
            blas = timeit(lambda: F.linear(x, w), a.iters)
            fl = 2.0 * m * n * k
            res = [f"{name:5s} M={m:5d}  blas {blas:7.1f}"]
            cands = []
            if m <= 128:
                for nt in (1, 2):
                    for sp in (1, 2, 4):
                        if n % (16 * nt) or k % ((256 if m > 64 else 512) * sp) or n % 64:
                            continue
                        cands.append((f"xc{nt}/{sp}", lambda nt=nt, sp=sp: ops.native().skinny_gemm(
                            x, wp, out, ws, sp, nt, -4), sp))
            for cfg in [int(c) for c in a.cfgs.split(",")]:
                bm, bn = {0: (256, 256), 1: (128, 256), 2: (256, 128), 3: (256, 256), 4: (256, 256),
                          5: (192, 256), 6: (192, 128), 10: (256, 256), 11: (192, 256),
                          12: (128, 256), 13: (256, 128), 14: (64, 256)}[cfg]
                tiles = -(-m // bm) * -(-n // bn)
                for sp in [int(v) for v in a.splits.split(",")]:
                    if k % (64 * sp) or (sp > 1 and tiles * sp > 2048) or (sp > 1 and tiles >= 512):
                        continue
                    cands.append((f"pg{cfg}/{sp}", lambda cfg=cfg, sp=sp: ops.native().packed_gemm(
                        x, wp, out, ws if sp > 1 else None, sp, 1 if sp > 1 else 0, cfg), sp))
            best = None
            xbest = None
            times = {}
            for label, fn, sp in cands:
                if sp > 1 and sp * m * n > ws.numel():
                    continue
                if sp > 1:
                    f = lambda fn=fn, sp=sp: (fn(), ops.slab_store(ws, sp, m, n, out))  # noqa: E731
                else:
                    f = fn
                f()
                torch.cuda.synchronize()
                err = (out.float() - ref).abs().max().item()
                if err > 0.1:
                    res.append(f"!!{label} err {err:.3f}")
                us = timeit(f, a.iters)
                times[label] = us
                if best is None or us < best[1]:
                    best = (label, us)
                if label.startswith("xc") and (xbest is None or us < xbest[1]):
                    xbest = (label, us)
            res.append(" ".join(f"{l}={t:.1f}" for l, t in sorted(times.items())))
            res.append(f"best {best[0]:9s} {best[1]:7.1f} us  {fl / best[1] / 1e6:6.0f} TF  "
                       f"vs blas {blas / best[1]:.2f}x")
            if xbest:
                res.append(f"(xc best {xbest[0]} {xbest[1]:.1f})")
            print("  ".join(res), flush=True)
        del w, wp, ws
        torch.cuda.empty_cache()
    n, k = 2 * 1024, 512
    w = torch.randn(n, k, device="cuda").bfloat16() * 0.05
    x = torch.randn(300, k, device="cuda").bfloat16()
    g, u = F.linear(x, w).float().chunk(2, dim=-1)
    for cfg in (0, 1, 3, 10, 11, 12, 13, 14):
        h = ops.packed_gemm(x, ops.pack_weight(ops.interleave_gate_up(w, 1)), epi="silu", cfg=cfg)
        print(f"silu epilogue cfg{cfg} max err",
              (h.float() - torch.nn.functional.silu(g) * u).abs().max().item())


if __name__ == "__main__":
    main()
