"""Sweep the fused-decode-layer GEMMs (csrc/kernels/skinny_pkr.hip) at Llama-3-8B
decode shapes, each in the epilogue the model runs it with, against hipBLASLt:

  qkv   store (split-K slabs for the RoPE kernel)
  o     resid (residual += y, in-launch split-K reduction)
  gu    silu + norm (RMSNorm + gate_up + SiLU-mul, one split)
  down  resid

From COLD caches: every call reads a different weight copy (copies total > 512
MB, past the 256 MB Infinity Cache); 32 calls are captured in one hipGraph.

python bench/pkr_sweep.py [--m 64] [--top 5]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402
from gemm_sweep import graph_time  # noqa: E402

SHAPES = {"qkv": (6144, 4096, "store"), "o": (4096, 4096, "resid"),
          "gu": (28672, 4096, "silu"), "down": (4096, 14336, "resid")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=64)
    ap.add_argument("--only", default="")
    ap.add_argument("--top", type=int, default=5)
    a = ap.parse_args()
    M = a.m
    dev = "cuda"
    torch.manual_seed(0)
    ws = torch.empty(16 * 64 * 6144, device=dev)
    tickets = torch.zeros(8192, dtype=torch.int32, device=dev)
    best = {}
    for name, (n, k, epi) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        ncopy = max(2, min(32, (640 << 20) // (n * k * 2)))
        Ws = [(torch.randn(n, k, device=dev) * 0.02).bfloat16() for _ in range(ncopy)]
        x = torch.randn(M, k, device=dev).bfloat16()
        calls = 32
        yo = torch.empty(M, n, device=dev).bfloat16()
        t_bl = graph_time([lambda W=Ws[i % ncopy]: torch.matmul(x, W.t(), out=yo)
                           for i in range(calls)])
        print(f"{name} M={M} N={n} K={k} epi={epi} copies={ncopy}: hipblaslt {t_bl:.2f} us "
              f"({n * k * 2 / t_bl / 1e3:.0f} GB/s)", flush=True)
        packed = {}

        def images(nt):
            key = nt if epi == "silu" else 0
            if key not in packed:
                packed.clear()
                packed[key] = [ops.pack_weight(ops.interleave_gate_up(w, nt // 2) if epi == "silu"
                                               else w) for w in Ws]
            return packed[key]
        rows = []
        res = torch.randn(M, n, device=dev).bfloat16()
        for nt, depth in ops.PKR_CONFIGS:
            if n % (16 * nt):
                continue
            if epi == "silu" and nt % 2:
                continue
            Wp = images(nt)
            for splits in ((1,) if epi == "silu" else (1, 2, 4, 8)):
                if k % (64 * splits) or (n // (16 * nt)) * splits < 96 or splits * M * n > ws.numel():
                    continue

                def f(W, nt=nt, sp=splits, d=depth):
                    if epi == "store":
                        return lambda: ops.pkr_gemm(x, W, "store", ws=ws, splits=sp, nt=nt, depth=d)
                    if epi == "resid":
                        return lambda: ops.pkr_gemm(x, W, "resid", residual=res, ws=ws, tickets=tickets,
                                                    splits=sp, nt=nt, depth=d)
                    return lambda: ops.pkr_gemm(x, W, "silu", nt=nt, depth=d, norm=True, eps=1e-5)
                # numerics of the plain GEMM part (store into slabs)
                if epi != "silu":
                    ops.pkr_gemm(x, Wp[0], "store", ws=ws, splits=splits, nt=nt, depth=depth)
                    got = ws[: splits * M * n].view(splits, M, n).sum(0)
                    err = (got - F.linear(x, Ws[0]).float()).abs().max().item()
                else:
                    err = 0.0
                t = graph_time([f(Wp[i % ncopy]) for i in range(calls)])
                rows.append((t, nt, depth, splits, err))
        rows.sort()
        for t, nt, depth, splits, err in rows[: a.top]:
            print(f"   nt={nt} depth={depth} splits={splits}: {t:7.2f} us "
                  f"({n * k * 2 / t / 1e3:5.0f} GB/s) err={err:.4f}", flush=True)
        bad = [r for r in rows if r[4] > 0.06]
        if bad:
            print("   !!! numerics failures:", bad[:3])
        best[name] = {"hipblaslt_us": round(t_bl, 2), "best": rows[0][:4] if rows else None}
        del Ws, Wp, packed
        torch.cuda.empty_cache()
    assert int(tickets.abs().sum().item()) == 0, "tickets not re-armed"
    print(json.dumps(best))


if __name__ == "__main__":
    main()
