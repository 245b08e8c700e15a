"""Post-attention half of a Llama-3-8B decode layer at 33..64 rows: the unfused launch
sequence (o xr -> add+RMSNorm -> gate_up xr+SiLU -> down xr -> add+RMSNorm, the
model's PACKED_PLAN at 64 rows) against the persistent decode block
(csrc/kernels/decode_block.hip), on NL distinct layers' weights cycled so every
layer streams from HBM (NL x 385 MB >> the 256 MiB Infinity Cache).

python bench/block_probe.py [--rows 50] [--layers 8] [--reps 20]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fasttalk_llm_microservice_amd import ops  # noqa: E402

H, KO, INTER, EPS = 4096, 4096, 14336, 1e-5


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[33, 50, 64])
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    ops.native()
    dev = "cuda"
    plan = ops.decode_block_plan(H, KO, INTER)
    print("plan (so, sd, tpw, grid):", plan)
    Ls = []
    for _ in range(a.layers):
        Ls.append(dict(wo=ops.pack_weight((torch.randn(H, KO, device=dev) * 0.02).bfloat16()),
                       wgu=ops.pack_weight((torch.randn(2 * INTER, H, device=dev) * 0.02).bfloat16()),
                       wd=ops.pack_weight((torch.randn(H, INTER, device=dev) * 0.02).bfloat16())))
    one = torch.ones(H, dtype=torch.bfloat16, device=dev)
    for m in a.rows:
        attn = torch.randn(m, KO, device=dev).bfloat16()
        res = torch.randn(m, H, device=dev).bfloat16()
        x = torch.empty(m, H, dtype=torch.bfloat16, device=dev)
        h = torch.empty(64, INTER, dtype=torch.bfloat16, device=dev)
        ws = torch.empty(max(4 * 64 * INTER, ops.decode_block_ws_floats(H, 64)), device=dev)
        xg = torch.empty(128 * 2 * 4 * 256, device=dev)
        ctl = torch.zeros(ops.decode_block_ctl_words(), dtype=torch.int32, device=dev)

        def unfused(L):
            ops.skinny_gemm(attn, L["wo"], ws=ws, splits=4, nt=1, u=-5)
            ops.row_rmsnorm(x, one, EPS, m, ws=ws, splits=4, residual=res)
            hh = ops.skinny_gemm(x, L["wgu"], splits=1, nt=2, u=-6)
            ops.skinny_gemm(hh, L["wd"], ws=ws, splits=4, nt=1, u=-5)
            ops.row_rmsnorm(x, one, EPS, m, ws=ws, splits=4, residual=res)

        def block(L):
            ops.decode_block(attn, res, h, L["wo"], L["wgu"], L["wd"], ws, xg, ctl, EPS)

        for name, fn in (("unfused", unfused), ("block", block), ("unfused", unfused), ("block", block)):
            for L in Ls:
                fn(L)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                for L in Ls:
                    fn(L)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / (a.reps * len(Ls))
            print(f"rows {m:3d} {name:8s} {us:7.1f} us/layer  ({385.9 / us:.2f} TB/s of weights)",
                  flush=True)
        print("ctl after:", int(ctl.abs().sum().item()), "err word:", int(ctl[2].item()), flush=True)
        # per-phase wall-clock stamps (100 MHz) of one layer launched between others
        st = torch.zeros(16 * 1024, dtype=torch.int64, device=dev)
        names = ["start", "O mma", "O seam", "bar1", "GU mma", "GU epi", "bar2", "D mma", "D seam"]
        acc = torch.zeros(len(names), 3, dtype=torch.float64)
        for rep in range(a.reps):
            for li, L in enumerate(Ls):
                ops.decode_block(attn, res, h, L["wo"], L["wgu"], L["wd"], ws, xg, ctl, EPS,
                                 stamps=st if li == len(Ls) // 2 else None)
            torch.cuda.synchronize()
            t = st.view(1024, 16)[:plan[3], :len(names)].double().cpu()
            t = (t - t[:, 0].min()) * 0.01   # us
            acc[:, 0] += t.min(0).values
            acc[:, 1] += t.mean(0)
            acc[:, 2] += t.max(0).values
        acc /= a.reps
        print(f"rows {m}: phase stamps, us from the first workgroup's start (min / mean / max over workgroups)")
        for k, n in enumerate(names):
            print(f"   {n:8s} {acc[k, 0]:7.2f} {acc[k, 1]:7.2f} {acc[k, 2]:7.2f}", flush=True)


if __name__ == "__main__":
    main()
