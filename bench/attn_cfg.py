"""Decode attention (fused combine, as the engine runs it) at the driver-config
shapes under env-selected kernel configurations (FT_DECODE_WPC / FT_DECODE_RING /
any FT_DECODE_* knob), cold KV (two copies alternate).  One process per config:
the knobs are read once per process.

python bench/attn_cfg.py "FT_DECODE_WPC=1 FT_DECODE_RING=2" "FT_DECODE_WPC=2 FT_DECODE_RING=2" ...
"""
import math
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "bench"))
    import torch

    from fasttalk_llm_microservice_amd import ops
    from gemm_sweep import graph_time

    nq, nkv, d, bs = 32, 8, 128, 16
    torch.manual_seed(0)
    res = []
    for B, ctx, uniform in [(50, 3000, False), (50, 4500, False), (64, 4096, True)]:
        nblk = math.ceil(ctx / bs)
        nblocks = B * nblk + 8
        kvs = [(torch.randn(nblocks, nkv, bs, d, device="cuda").bfloat16(),
                torch.randn(nblocks, nkv, d, bs, device="cuda").bfloat16()) for _ in range(2)]
        bt = torch.randperm(nblocks, device="cuda")[: B * nblk].int().view(B, nblk)
        sl = torch.full((B,), ctx, dtype=torch.int32, device="cuda") if uniform else \
            torch.randint(ctx // 2, ctx + 1, (B,), dtype=torch.int32, device="cuda")
        q = torch.randn(B, (nq + 2 * nkv) * d, device="cuda").bfloat16()
        out = torch.empty(B, nq * d, device="cuda").bfloat16()
        n_out, n_ml = ops.decode_workspace(B, nq, nkv, d)
        to, tm = torch.empty(n_out, device="cuda"), torch.empty(n_ml, device="cuda")
        cnt = ops.decode_counters(B, nkv, "cuda")
        nbytes = int(sl.sum().item()) * nkv * d * 4
        t = graph_time([lambda kv=kvs[i % 2]: ops.decode_attention(out, q, kv[0], kv[1], bt, sl, to, tm, nq, nkv,
                                                                   d, d ** -0.5, counters=cnt) for i in range(8)])
        res.append(f"B={B} ctx={ctx}{'u' if uniform else ''}: {t:6.1f} us {nbytes / t / 1e3:5.0f} GB/s")
        del kvs
        torch.cuda.empty_cache()
    print("   " + " | ".join(res), flush=True)


def main():
    if os.environ.get("ATTN_CFG_CHILD"):
        return child()
    for spec in sys.argv[1:] or [""]:
        env = dict(os.environ, ATTN_CFG_CHILD="1")
        for kv in spec.split():
            k, v = kv.split("=", 1)
            env[k] = v
        print(f"[{spec or 'default'}]", flush=True)
        r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, timeout=300)
        if r.returncode != 0:
            print(f"   failed rc={r.returncode}", flush=True)
            if r.returncode < 0 or r.returncode > 1:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
