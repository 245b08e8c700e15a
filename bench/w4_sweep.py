"""Sweep the W4A16 decode GEMM (csrc/kernels/w4a16.hip) over (nt, splits) at the
Llama-3-8B projection shapes and decode row counts, from cold caches (distinct
weight copies > the 256 MB MALL, 32 calls per hipGraph), against the bf16 packed
kernel plan and hipBLASLt on bf16 weights.  Checks numerics of every config.

python bench/w4_sweep.py [--ms 1,8,16,32,64] [--shapes name:N:K,...]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from gemm_sweep import graph_time  # noqa: E402
from fasttalk_llm_microservice_amd.ops import quant as Q  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,8,16,32,64")
    ap.add_argument("--shapes", default="qkv:6144:4096,o:4096:4096,gu:28672:4096,down:4096:14336")
    ap.add_argument("--top", type=int, default=4)
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    ws = torch.empty(8 * 64 * 28672, device=dev)
    for spec in a.shapes.split(","):
        name, n, k = spec.split(":")
        n, k = int(n), int(k)
        w = torch.randn(n, k, device=dev) * 0.02
        q, z, s = Q.quantize_w4(w)
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
            for nt in (1, 2, 4):
                for sp in (1, 2, 4, 8):
                    if n % (16 * nt) or k % (128 * sp) or sp * m * n > ws.numel():
                        continue
                    if (n // (16 * nt)) * sp < 128:
                        continue
                    if sp == 1:
                        fn = lambda W, nt=nt: (lambda: Q.w4_gemm(x, W, out=out, nt=nt))
                        fn(W0)()
                        y = out.float()
                    else:
                        fn = lambda W, nt=nt, sp=sp: (lambda: Q.w4_gemm(x, W, ws=ws, splits=sp, nt=nt))
                        fn(W0)()
                        y = ws[:sp * m * n].view(sp, m, n).sum(0)
                    err = (y - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
                    try:
                        t = graph_time([fn(W) for W in seq])
                    except RuntimeError as e:  # unsupported tile count for this M
                        print(f"  skip nt={nt} sp={sp}: {e}")
                        continue
                    rows.append((t, nt, sp, err))
            rows.sort()
            best = ", ".join(f"nt{nt}/s{sp} {t:.2f}us (err {e:.1e})" for t, nt, sp, e in rows[:a.top])
            gbs = W0.nbytes() / rows[0][0] / 1e3 if rows else 0
            print(f"{name} N={n} K={k} M={m}: {best}  -> {gbs:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
