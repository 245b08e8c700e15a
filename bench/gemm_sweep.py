"""Sweep skinny_gemm configs (both variants) at decode shapes vs hipBLASLt from
COLD caches: every call reads a different copy of the weight (copies total
> 512 MB, beyond the 256 MB MALL), and 32 calls are captured in one hipGraph so
launch overhead is not measured.  Checks numerics of every config.

python bench/gemm_sweep.py [--m 50] [--shapes name:N:K,...]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402


def graph_time(fn_list, reps=5):
    """us per call of a list of thunks captured in one hipGraph."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for f in fn_list[:2]:
            f()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for f in fn_list:
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * len(fn_list))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=50)
    ap.add_argument("--shapes", default="qkv:6144:4096,o:4096:4096,gate_up:28672:4096,"
                                        "down:4096:14336,lm_head:128256:4096")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    M = a.m
    dev = "cuda"
    torch.manual_seed(0)
    best = {}
    ws = torch.empty(32 * 64 * 28672, device=dev)
    for spec in a.shapes.split(","):
        name, n, k = spec.split(":")
        n, k = int(n), int(k)
        ncopy = max(2, min(32, (640 << 20) // (n * k * 2)))
        Ws = [(torch.randn(n, k, device=dev) * 0.02).bfloat16() for _ in range(ncopy)]
        x = torch.randn(M, k, device=dev).bfloat16()
        ref = F.linear(x, Ws[0]).float()
        calls = 32
        seqW = [Ws[i % ncopy] for i in range(calls)]
        yo = torch.empty(M, n, device=dev).bfloat16()
        t_bl = graph_time([lambda W=W: torch.matmul(x, W.t(), out=yo) for W in seqW])
        print(f"{name} N={n} K={k} copies={ncopy}: hipblaslt {t_bl:.2f} us "
              f"({n * k * 2 / t_bl / 1e3:.0f} GB/s)", flush=True)
        rows = []
        out = torch.empty(M, n, device=dev).bfloat16()
        for nt, u in ops.SKINNY_CONFIGS:
            for splits in (1, 2, 4, 8, 16):
                kstep = (512 if u == -4 else 64) * splits
                if n % (16 * nt) or k % kstep or splits * M * n > ws.numel():
                    continue
                cols = 16 * nt if u == -3 else 64 * nt
                blocks = (n // cols) * splits
                if blocks < 128 or blocks > 16384:
                    continue
                if splits == 1:
                    mk = lambda W, nt=nt, u=u: (lambda: ops.skinny_gemm(x, W, out=out, nt=nt, u=u))
                else:
                    mk = lambda W, nt=nt, u=u, sp=splits: (
                        lambda: ops.skinny_gemm(x, W, ws=ws, splits=sp, nt=nt, u=u))
                if u in ops.PACKED_VARIANTS:  # pre-packed weights
                    packed = [ops.pack_weight(W) for W in Ws]
                    mk0 = mk
                    mk = lambda W, mk0=mk0, packed=packed: mk0(packed[[id(x) for x in Ws].index(id(W))])
                f0 = mk(Ws[0])
                f0()
                torch.cuda.synchronize()
                got = out.float() if splits == 1 else ws[: splits * M * n].view(splits, M, n).sum(0)
                err = (got - ref).abs().max().item()
                t = graph_time([mk(W) for W in seqW])
                rows.append((t, nt, u, splits, blocks, err))
                if u in ops.PACKED_VARIANTS:
                    del packed
        rows.sort()
        for t, nt, u, splits, blocks, err in rows[: a.top]:
            print(f"   {({-3: 'pk', -4: 'xcp'}).get(u, '?')} nt={nt} u={u} splits={splits:2d} blocks={blocks:5d}: "
                  f"{t:7.2f} us ({n * k * 2 / t / 1e3:5.0f} GB/s) err={err:.4f}", flush=True)
        bad = [r for r in rows if r[5] > 0.05]
        if bad:
            print("   !!! numerics failures:", bad[:3])
        best[name] = {"hipblaslt_us": round(t_bl, 2), "best": rows[0][:5] if rows else None}
        del Ws
        torch.cuda.empty_cache()
    print(json.dumps(best))


if __name__ == "__main__":
    main()
