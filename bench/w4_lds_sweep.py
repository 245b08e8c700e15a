"""W4A16 decode GEMMs at 17..64 rows (w4a16.hip): the register kernel, "xr" (x chunks
in LDS) and "mh" (two tiles per wave, rows over wave pairs; ring 2 with two x chunks
in flight = xr 4, ring 3 = xr 5) against the model's plan entry (w4_cfg), cold caches
(distinct weight copies, 32 calls per hipGraph), at the Llama-3-8B projection shapes;
gate_up also with the SiLU epilogues.  Checks every config's numerics against the
fp32 product of the dequantized weights.

python bench/w4_lds_sweep.py [--ms 33,50,64] [--shapes gu:28672:4096,...]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gemm_sweep import graph_time  # noqa: E402
from fasttalk_llm_microservice_amd.models.llama import w4_cfg, w4_fits  # noqa: E402
from fasttalk_llm_microservice_amd.ops import quant as Q  # noqa: E402

NAMES = {0: "reg", 1: "xr", 4: "mh", 5: "mh3"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="33,50,64")
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
            cfgs = [("plan",) + tuple(w4_cfg(name, m, n, k))]
            for sp in (1, 2, 4, 7, 8, 14):
                cfgs += [("reg", 4, sp, 0), ("xr", 2, sp, 1), ("mh", 2, sp, 4), ("mh3", 2, sp, 5)]
            for kind, nt, sp, xr in cfgs:
                if not w4_fits(xr, nt, sp, n, k) or sp * m * n > ws.numel():
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
                rows.append((graph_time([fn(W) for W in seq]), kind, nt, sp, err))
            if name == "gu":   # SiLU epilogues (16-column gate / up pairs)
                g_, u_ = ref.view(m, -1, 2, 16).unbind(2)
                href = (torch.nn.functional.silu(g_) * u_).reshape(m, -1)
                hout = torch.empty(m, n // 2, device=dev).bfloat16()
                for xr in (1, 4, 5):
                    if not w4_fits(xr, 2, 1, n, k):
                        continue
                    fn = lambda W, xr=xr: (lambda: Q.w4_gemm(x, W, out=hout, nt=2, xr=xr, silu=True))
                    fn(W0)()
                    err = (hout.float() - href).abs().max().item() / (href.abs().max().item() + 1e-6)
                    rows.append((graph_time([fn(W) for W in seq]), NAMES[xr] + "-silu", 2, 1, err))
            rows.sort()
            best = "  ".join(f"{kd}{nt}/{sp}={t:.1f}" + (f"(ERR {e:.0e})" if e > 2e-2 else "")
                             for t, kd, nt, sp, e in rows)
            print(f"{name} N={n} K={k} M={m} [{W0.nbytes() / rows[0][0] / 1e3:.0f} GB/s best] "
                  f"maxerr {max(r[4] for r in rows):.1e}: {best}", flush=True)


if __name__ == "__main__":
    main()
