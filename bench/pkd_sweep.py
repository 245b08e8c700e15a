"""Cold-cache sweep of the deep-ring packed decode GEMM (skinny_pkd_kernel, u=-5)
against the current PACKED_PLAN kernel per projection, at the decode bucket of
64 rows (M = 50 real rows): every call reads a different copy of the packed
weight (copies > 512 MB, beyond the 256 MB MALL) and 32 calls are captured in
one hipGraph.  Numerics of every config are checked against hipBLASLt.

python bench/pkd_sweep.py [--m 50] [--shapes qkv:6144:4096,...]
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
from fasttalk_llm_microservice_amd.models import llama  # noqa: E402
from gemm_sweep import graph_time  # noqa: E402

PLAN_KEY = {"qkv": "qkv", "o": "o", "gate_up": "gu", "down": "down", "lm_head": "lm"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=50)
    ap.add_argument("--shapes", default="qkv:6144:4096,o:4096:4096,gate_up:28672:4096,"
                                        "down:4096:14336,lm_head:128256:4096")
    ap.add_argument("--top", type=int, default=6)
    a = ap.parse_args()
    M = a.m
    dev = "cuda"
    torch.manual_seed(0)
    ws = torch.empty(16 * 64 * 28672, device=dev)
    summary = {}
    for spec in a.shapes.split(","):
        name, n, k = spec.split(":")
        n, k = int(n), int(k)
        ncopy = max(2, min(32, (640 << 20) // (n * k * 2)))
        Ws = [(torch.randn(n, k, device=dev) * 0.02).bfloat16() for _ in range(ncopy)]
        P = [ops.pack_weight(W) for W in Ws]
        x = torch.randn(M, k, device=dev).bfloat16()
        ref = F.linear(x, Ws[0]).float()
        calls = 32
        seq = [i % ncopy for i in range(calls)]
        out = torch.empty(M, n, device=dev).bfloat16()
        yo = torch.empty(M, n, device=dev).bfloat16()
        t_bl = graph_time([lambda i=i: torch.matmul(x, Ws[i].t(), out=yo) for i in seq])
        rows = []
        plan = llama.packed_cfg(PLAN_KEY[name], M)
        cands = []
        if plan is not None:
            nt, u, sp = plan
            cands.append(("plan", nt, u, sp, 0))
        for nt in (1, 2, 4):
            for depth in (2, 4, 6):
                if nt == 4 and depth == 6:
                    continue
                for sp in (1, 2, 4, 8):
                    if n % (16 * nt) or k % (64 * sp) or sp * M * n > ws.numel():
                        continue
                    blocks = (n // (16 * nt)) * sp
                    if blocks < 128 or blocks > 8192:
                        continue
                    cands.append(("pkd", nt, -5, sp, depth))
        for kind, nt, u, sp, depth in cands:
            def mk(i, nt=nt, u=u, sp=sp, depth=depth):
                if sp == 1:
                    return lambda: ops.skinny_gemm(x, P[i], out=out, nt=nt, u=u, depth=depth or 4)
                return lambda: ops.skinny_gemm(x, P[i], ws=ws, splits=sp, nt=nt, u=u, depth=depth or 4)
            mk(0)()
            torch.cuda.synchronize()
            got = out.float() if sp == 1 else ws[: sp * M * n].view(sp, M, n).sum(0)
            err = (got - ref).abs().max().item()
            t = graph_time([mk(i) for i in seq])
            rows.append((t, kind, nt, sp, depth, err))
        rows.sort()
        planrow = [r for r in rows if r[1] == "plan"]
        print(f"{name} N={n} K={k}: hipblaslt {t_bl:.2f} us; plan "
              f"{planrow[0][0] if planrow else float('nan'):.2f} us", flush=True)
        for t, kind, nt, sp, depth, err in rows[: a.top]:
            print(f"   {kind} nt={nt} splits={sp} depth={depth}: {t:7.2f} us "
                  f"({n * k * 2 / t / 1e3:5.0f} GB/s) err={err:.4f}", flush=True)
        bad = [r for r in rows if r[5] > 0.05]
        if bad:
            print("   !!! numerics failures:", bad[:3])
        summary[name] = {"hipblaslt_us": round(t_bl, 2),
                         "plan_us": round(planrow[0][0], 2) if planrow else None,
                         "best": [round(rows[0][0], 2)] + list(rows[0][1:5])}
        del Ws, P
        torch.cuda.empty_cache()
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
