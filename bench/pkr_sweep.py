"""Sweep the fused-decode-layer GEMMs (csrc/kernels/skinny_pkr.hip) at Llama-3-8B
decode shapes, each in the epilogue the model runs it with, against hipBLASLt:

  qkv   store (split-K slabs for the RoPE kernel)
  o     resid (residual += y, in-launch split-K reduction)
  gu    silu + norm (RMSNorm + gate_up + SiLU-mul, one split)
  down  resid

From COLD caches: every call reads a different weight copy (copies total > 512
MB, past the 256 MB Infinity Cache); 32 calls are captured in one hipGraph.
``--plan-out`` writes the fastest (nt, depth, splits) per projection and row
count as the model's fused_plan.json (gate_up: the one nt that is fastest summed
over the row counts, since the interleaved packing fixes it).

python bench/pkr_sweep.py [--m 64,32,16,8,1] [--top 5] [--plan-out PATH]
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
CALLS = 32


def sweep_shape(n, k, epi, Ms, ws, tickets):
    ncopy = max(2, min(32, (640 << 20) // (n * k * 2)))
    Ws = [(torch.randn(n, k, device="cuda") * 0.02).bfloat16() for _ in range(ncopy)]
    xs = {M: torch.randn(M, k, device="cuda").bfloat16() for M in Ms}
    ress = {M: torch.randn(M, n, device="cuda").bfloat16() for M in Ms}
    bl = {}
    for M in Ms:
        yo = torch.empty(M, n, device="cuda").bfloat16()
        bl[M] = graph_time([lambda W=Ws[i % ncopy], x=xs[M]: torch.matmul(x, W.t(), out=yo)
                            for i in range(CALLS)])
    rows = {M: [] for M in Ms}
    packed_key, Wp = None, None
    for nt, depth in ops.PKR_CONFIGS:
        if n % (16 * nt) or (epi == "silu" and nt % 2):
            continue
        key = nt if epi == "silu" else 0
        if key != packed_key:
            Wp = None
            torch.cuda.empty_cache()
            Wp = [ops.pack_weight(ops.interleave_gate_up(w, nt // 2) if epi == "silu" else w)
                  for w in Ws]
            packed_key = key
        for M in Ms:
            x, res = xs[M], ress[M]
            for sp in ((1,) if epi == "silu" else (1, 2, 4, 8)):
              for wn in ((False, True) if M > 32 and n % (64 * nt) == 0 else (False,)):
                if k % (64 * sp) or sp * M * n > ws.numel():
                    continue

                def f(W, nt=nt, sp=sp, d=depth, x=x, res=res, wn=wn):
                    if epi == "store":
                        return lambda: ops.pkr_gemm(x, W, "store", ws=ws, splits=sp, nt=nt, depth=d,
                                                    wn=wn)
                    if epi == "resid":
                        return lambda: ops.pkr_gemm(x, W, "resid", residual=res, ws=ws, tickets=tickets,
                                                    splits=sp, nt=nt, depth=d, wn=wn)
                    return lambda: ops.pkr_gemm(x, W, "silu", nt=nt, depth=d, norm=True, eps=1e-5,
                                                wn=wn)
                err = 0.0
                if epi != "silu":  # numerics of the GEMM part (slabs)
                    ops.pkr_gemm(x, Wp[0], "store", ws=ws, splits=sp, nt=nt, depth=depth, wn=wn)
                    got = ws[: sp * M * n].view(sp, M, n).sum(0)
                    err = (got - F.linear(x, Ws[0]).float()).abs().max().item()
                t = graph_time([f(Wp[i % ncopy]) for i in range(CALLS)])
                rows[M].append((t, nt, depth, sp, int(wn), err))
    del Ws, Wp
    torch.cuda.empty_cache()
    return bl, rows


def make_plan(results):
    plan = {}
    for name, per in results.items():
        if name == "gu":
            nts = sorted({r[1] for rs in per.values() for r in rs})

            def total(nt):
                return sum(min((r[0] for r in rs if r[1] == nt), default=1e9) for rs in per.values())
            nt_best = min(nts, key=total)
            per = {M: [r for r in rs if r[1] == nt_best] for M, rs in per.items()}
        plan[name] = {str(M): list(min(rs)[1:5]) for M, rs in per.items() if rs}
    return plan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="64")
    ap.add_argument("--only", default="")
    ap.add_argument("--top", type=int, default=5)
    ap.add_argument("--plan-out", default="")
    a = ap.parse_args()
    Ms = [int(v) for v in a.m.split(",")]
    torch.manual_seed(0)
    ws = torch.empty(8 * 64 * 6144, device="cuda")
    tickets = torch.zeros(8192, dtype=torch.int32, device="cuda")
    results, summary = {}, {}
    for name, (n, k, epi) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        bl, rows = sweep_shape(n, k, epi, Ms, ws, tickets)
        results[name] = rows
        for M in Ms:
            rs = sorted(rows[M])
            print(f"{name} M={M} N={n} K={k} epi={epi}: hipblaslt {bl[M]:.2f} us "
                  f"({n * k * 2 / bl[M] / 1e3:.0f} GB/s)", flush=True)
            for t, nt, depth, sp, wn, err in rs[: a.top]:
                print(f"   nt={nt} depth={depth} splits={sp} wn={wn}: {t:7.2f} us "
                      f"({n * k * 2 / t / 1e3:5.0f} GB/s) err={err:.4f}", flush=True)
            bad = [r for r in rs if r[5] > 0.06]
            if bad:
                print("   !!! numerics failures:", bad[:3], flush=True)
            summary.setdefault(name, {})[M] = {"hipblaslt_us": round(bl[M], 2),
                                               "best": [round(rs[0][0], 2)] + list(rs[0][1:5])}
    assert int(tickets.abs().sum().item()) == 0, "tickets not re-armed"
    print(json.dumps(summary))
    if a.plan_out:
        plan = make_plan(results)
        with open(a.plan_out, "w") as f:
            json.dump(plan, f, indent=1)
        print("plan:", json.dumps(plan))


if __name__ == "__main__":
    main()
