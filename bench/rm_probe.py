"""A/B of the decode GEMM kernels on the packed MFMA-fragment image vs the same
kernels reading row-major W[N, K] (u = -13 / -14), cold cache (weights rotated
through > 512 MiB so neither L2 nor the 256 MiB MALL holds them), at the
Llama-3-8B projection shapes and decode row counts.  Decides whether the model
can keep ONE weight image (row-major, shared with hipBLASLt prefill GEMMs).

python bench/rm_probe.py [--rows 1,8,16,32,50,64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (28672, 4096), "down": (4096, 14336),
          "lm": (128256, 4096)}
CONFIGS = [(1, -3, 1), (2, -3, 1), (4, -3, 1), (2, -3, 2), (4, -3, 4), (2, -3, 4), (1, -4, 1),
           (2, -4, 1), (2, -4, 2), (1, -4, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="1,8,16,32,50,64")
    ap.add_argument("--only", default="")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--configs", default="", help="nt:u:splits,... (default: the built-in list)")
    ap.add_argument("--packed-only", action="store_true")
    a = ap.parse_args()
    rows = [int(r) for r in a.rows.split(",")]
    configs = [tuple(int(v) for v in c.split(":")) for c in a.configs.split(",")] if a.configs \
        else CONFIGS
    res = {}
    torch.manual_seed(0)
    for name, (n, k) in SHAPES.items():
        if a.only and name not in a.only.split(","):
            continue
        nbytes = n * k * 2
        copies = max(2, -(-(600 << 20) // nbytes))
        ws_rm = [torch.randn(n, k, device="cuda").bfloat16() * 0.02 for _ in range(copies)]
        ws_pk = [ops.pack_weight(w) for w in ws_rm]
        ws = torch.empty(16 * 64 * max(n, 4096), device="cuda")
        for m in rows:
            x = torch.randn(m, k, device="cuda").bfloat16()
            ref = F.linear(x, ws_rm[0]).float()
            best = {}
            per_cfg = {}
            for nt, u, sp in configs:
                kq = {-4: 512, -5: 512 if nt == 2 else 256, -6: 512}.get(u, 64)
                if n % (16 * nt) or k % (kq * sp) or (u == -4 and n % 64):
                    continue
                if u == -6 and (sp != 1 or nt != 2 or name != "gu"):
                    continue
                for rm in ((False,) if a.packed_only or u <= -5 else (False, True)):
                    uu = u - 10 if rm else u
                    imgs = ws_rm if rm else ws_pk
                    out = torch.empty(m, n // 2 if u == -6 else n, device="cuda").bfloat16()

                    def run(i):
                        ops.native().skinny_gemm(x, imgs[i % copies], out, ws, sp, nt, uu)
                    if sp == 1:
                        run(0)
                        r = ref
                        if u == -6:  # gate/up interleaved in 16-column groups -> silu(g) * u
                            r4 = ref.view(m, n // 32, 2, 16)
                            r = (F.silu(r4[:, :, 0]) * r4[:, :, 1]).reshape(m, n // 2)
                        err = (out.float() - r).abs().max().item()
                        if err > 0.05:
                            print(f"  !! {name} m={m} nt={nt} u={uu} err {err}", flush=True)
                    for i in range(5):
                        run(i)
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for i in range(a.iters):
                        run(i)
                    e.record()
                    torch.cuda.synchronize()
                    us = s.elapsed_time(e) * 1e3 / a.iters
                    key = "rm" if rm else "pk"
                    if not rm:
                        per_cfg[(nt, u, sp)] = us
                    if key not in best or us < best[key][0]:
                        best[key] = (us, (nt, u, sp))
            # hipBLASLt on the row-major copies
            for i in range(5):
                F.linear(x, ws_rm[i % copies])
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i in range(a.iters):
                F.linear(x, ws_rm[i % copies])
            e.record()
            torch.cuda.synchronize()
            blas = s.elapsed_time(e) * 1e3 / a.iters
            if a.packed_only:
                print(f"{name:5s} m={m:3d} blas {blas:6.2f} " + " ".join(
                    f"{c[0]}/{c[1]}/{c[2]}={t:.1f}" for c, t in sorted(per_cfg.items(), key=lambda kv: kv[1])),
                    flush=True)
                continue
            pk, rm = best.get("pk", (0, None)), best.get("rm", (0, None))
            line = (f"{name:5s} m={m:3d}  packed {pk[0]:7.2f} us {str(pk[1]):14s} "
                    f"row-major {rm[0]:7.2f} us {str(rm[1]):14s} hipblaslt {blas:7.2f} us  "
                    f"rm/pk {rm[0] / pk[0]:.3f}  rm {nbytes / rm[0] / 1e3:6.0f} GB/s")
            print(line, flush=True)
            res[f"{name}/{m}"] = {"pk": pk, "rm": rm, "blas": blas}
        del ws_rm, ws_pk
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
