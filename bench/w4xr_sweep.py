"""W4A16 decode GEMMs at 33..64 rows: the x-in-LDS "xr" variant (nt, splits) vs the
register kernel (w4a16.hip), cold caches (distinct weight copies, 32 calls per
hipGraph), at the Llama-3-8B projection shapes; gate_up with the SiLU epilogue.
Checks numerics of every config.

python bench/w4xr_sweep.py [--ms 50,64]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gemm_sweep import graph_time  # noqa: E402
from fasttalk_llm_microservice_amd.ops import quant as Q  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="50,64")
    ap.add_argument("--shapes", default="qkv:6144:4096,o:4096:4096,gu:28672:4096,down:4096:14336")
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    ws = torch.empty(16 * 64 * 28672, device=dev)
    for spec in a.shapes.split(","):
        name, n, k = spec.split(":")
        n, k = int(n), int(k)
        q, z, s = Q.quantize_w4(torch.randn(n, k, device=dev) * 0.02)
        W0 = Q.pack_w4(q, z, s)
        wdq = Q.dequantize_w4(q, z, s)
        ncopy = max(2, min(32, (640 << 20) // W0.nbytes()))
        Ws = [W0] + [Q.W4Weight(W0.wq.clone(), W0.sz.clone(), n, k) for _ in range(ncopy - 1)]
        seq = [Ws[i % ncopy] for i in range(32)]
        for m in [int(v) for v in a.ms.split(",")]:
            x = torch.randn(m, k, device=dev).bfloat16()
            ref = x.float() @ wdq.t()
            out = torch.empty(m, n, device=dev).bfloat16()
            rows = []
            cfgs = [("reg", nt, sp) for nt in (2, 4) for sp in (1, 2, 4, 8)] + \
                   [("xr", nt, sp) for nt in (1, 2, 4) for sp in (1, 2, 4, 7, 8, 14)] + \
                   [("xr8", 1, sp) for sp in (1, 2, 4, 7, 8)] + \
                   [("xrm", nt, sp) for nt in (1, 2) for sp in (1, 2, 4, 7, 8)]
            for kind, nt, sp in cfgs:
                xr = {"reg": 0, "xr": 1, "xr8": 2, "xrm": 3}[kind]
                kq = 512 if xr else 128
                if n % ((64 if xr else 16) * nt) or k % (kq * sp) or sp * m * n > ws.numel():
                    continue
                if sp == 1:
                    fn = lambda W, nt=nt, xr=xr: (lambda: Q.w4_gemm(x, W, out=out, nt=nt, xr=xr))
                    fn(W0)()
                    y = out.float()
                else:
                    fn = lambda W, nt=nt, sp=sp, xr=xr: (lambda: Q.w4_gemm(x, W, ws=ws, splits=sp, nt=nt, xr=xr))
                    fn(W0)()
                    y = ws[:sp * m * n].view(sp, m, n).sum(0)
                err = (y - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
                try:
                    t = graph_time([fn(W) for W in seq])
                except RuntimeError as e:
                    print(f"  skip {kind} nt={nt} sp={sp}: {e}")
                    continue
                rows.append((t, kind, nt, sp, err))
            if name == "gu":   # the xr SiLU epilogue (interleaved image; time only)
                hout = torch.empty(m, n // 2, device=dev).bfloat16()
                fn = lambda W: (lambda: Q.w4_gemm(x, W, out=hout, nt=2, xr=True, silu=True))
                rows.append((graph_time([fn(W) for W in seq]), "xr-silu", 2, 1, 0.0))
                fn = lambda W: (lambda: Q.w4_gemm(x, W, out=hout, nt=1, xr=2, silu=True))
                rows.append((graph_time([fn(W) for W in seq]), "xr8-silu", 2, 1, 0.0))
                fn = lambda W: (lambda: Q.w4_gemm(x, W, out=hout, nt=2, xr=3, silu=True))
                rows.append((graph_time([fn(W) for W in seq]), "xrm-silu", 2, 1, 0.0))
            rows.sort()
            best = "  ".join(f"{kd}{nt}/{sp}={t:.1f}" + (f"(err {e:.0e})" if e > 2e-2 else "")
                             for t, kd, nt, sp, e in rows)
            print(f"{name} N={n} K={k} M={m} [{W0.nbytes() / rows[0][0] / 1e3:.0f} GB/s best]: {best}", flush=True)


if __name__ == "__main__":
    main()
