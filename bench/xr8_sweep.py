"""4-wave vs 8-wave "xr" decode GEMM workgroups (skinny_gemm u = -5/-6 vs -7/-8)
at the Llama-3-8B projection shapes and 50 / 64 rows, cold weights (copies >
MALL), 32 calls per hipGraph; numerics checked against fp32.

python bench/xr8_sweep.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402
from gemm_sweep import graph_time  # noqa: E402


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="8b", choices=["8b", "70b"])
    ap.add_argument("--rows", default="50,64")
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = "cuda"
    if a.model == "70b":   # Llama-3-70B at TP=1: H 8192, I 28672, 64 q / 8 kv heads
        shapes = [("qkv", 10240, 8192, False), ("o", 8192, 8192, False), ("gu", 57344, 8192, True),
                  ("down", 8192, 28672, False)]
    else:
        shapes = [("qkv", 6144, 4096, False), ("o", 4096, 4096, False), ("gu", 28672, 4096, True),
                  ("down", 4096, 14336, False)]
    ws = torch.empty(8 * 64 * max(n for _, n, _, _ in shapes), device=dev)
    for name, n, k, gu in shapes:
        ncopy = max(2, min(32, (640 << 20) // (n * k * 2)))
        Wr = [(torch.randn(n, k, device=dev) * 0.02).bfloat16() for _ in range(ncopy)]
        if gu:
            Wr = [ops.interleave_gate_up(w, 1) for w in Wr]
        Wp = [ops.pack_weight(w) for w in Wr]
        for M in [int(r) for r in a.rows.split(",")]:
            x = torch.randn(M, k, device=dev).bfloat16()
            ref = (x.float() @ Wr[0].float().t())
            if gu:
                g, u = ref.view(M, n // 32, 2, 16).unbind(2)
                ref = (torch.nn.functional.silu(g) * u).reshape(M, n // 2)
            res = []
            for u in ((-6, -8) if gu else (-5, -7)):
                for nt in ((2,) if gu else (1, 2)):
                    kc = 512 if nt == 2 else 256
                    nw = 8 if u <= -7 else 4
                    for sp in ((1,) if gu else (1, 2, 4, 7, 8)):
                        if k % (kc * sp) or n % (16 * nt * nw) or sp * M * n > ws.numel():
                            continue
                        if sp == 1:
                            out = torch.empty(M, n // 2 if gu else n, device=dev).bfloat16()
                            fns = [lambda W=W: ops.skinny_gemm(x, W, out=out, nt=nt, u=u)
                                   for W in (Wp[i % ncopy] for i in range(32))]
                        else:
                            fns = [lambda W=W: ops.skinny_gemm(x, W, ws=ws, splits=sp, nt=nt, u=u)
                                   for W in (Wp[i % ncopy] for i in range(32))]
                        t = graph_time(fns)
                        fns[0]()
                        torch.cuda.synchronize()
                        y = out.float() if sp == 1 else ws[: sp * M * n].view(sp, M, n).sum(0)
                        err = (y - ref).abs().max().item() / ref.abs().max().item()
                        res.append((t, f"w{nw}/nt{nt}/s{sp}={t:.1f}" + ("" if err < 2e-2 else f"(ERR {err:.2e})")))
            res.sort()
            print(f"{name} N={n} K={k} M={M} [{n * k * 2 / res[0][0] / 1e3:.0f} GB/s best]: "
                  + "  ".join(r for _, r in res), flush=True)
        del Wr, Wp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
