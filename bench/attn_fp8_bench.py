"""Decode attention on fp8 (e4m3) vs bf16 KV caches at the serving shapes: 50 / 64
sequences with ragged 1.5-4.5k contexts, GQA 4 (Llama-3-8B), cold caches (several
KV copies alternate inside one hipGraph).  Prints us per call and the KV bytes
streamed per second.  FT_DECODE_RING8 (read once per process) picks the fp8 ring.

python bench/attn_fp8_bench.py
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402
from gemm_sweep import graph_time  # noqa: E402

nq, nkv, d = 32, 8, 128
bs = int(os.environ.get("BS", "16"))   # KV block size (tokens)


def main():
    g = torch.Generator().manual_seed(0)
    for B, lo, hi in [(50, 1500, 3000), (50, 2200, 4500), (64, 4096, 4097)]:
        lens = torch.randint(lo, hi, (B,), generator=g).tolist()
        nblk = [math.ceil(n / bs) for n in lens]
        total = sum(nblk)
        bt = torch.zeros(B, max(nblk), dtype=torch.int32)
        perm = torch.randperm(total + 8, generator=g).int()
        o = 0
        for i, n in enumerate(nblk):
            bt[i, :n] = perm[o:o + n]
            o += n
        bt, sl = bt.cuda(), torch.tensor(lens, dtype=torch.int32, device="cuda")
        q = torch.randn(B, nq * d, device="cuda").bfloat16()
        n_out, n_ml = ops.decode_workspace(B, nq, nkv, d)
        tmp = (torch.empty(n_out, device="cuda"), torch.empty(n_ml, device="cuda"))
        cnt = ops.decode_counters(B, nkv, "cuda")
        out = torch.empty(B, nq * d, device="cuda").bfloat16()
        res = {}
        for name, dt in (("bf16", torch.bfloat16), ("fp8", torch.float8_e4m3fn)):
            ncopy = 3 if dt == torch.bfloat16 else 6
            kvs = []
            for _ in range(ncopy):
                k = torch.randn(total + 8, nkv, bs, d, device="cuda").to(dt)
                v = torch.randn(total + 8, nkv, d, bs, device="cuda").to(dt)
                kvs.append((k, v))
            fns = [(lambda k=k, v=v: ops.decode_attention(out, q, k, v, bt, sl, tmp[0], tmp[1], nq, nkv, d,
                                                          d ** -0.5, counters=cnt)) for k, v in kvs] * 4
            us = graph_time(fns)
            nbytes = sum(lens) * nkv * d * 2 * kvs[0][0].element_size()
            res[name] = us
            print(f"B={B} ctx {lo}-{hi}: {name} {us:.1f} us, {nbytes / us / 1e6:.2f} TB/s of KV", flush=True)
            del kvs, fns
            torch.cuda.empty_cache()
        print(f"B={B} ctx {lo}-{hi}: fp8 / bf16 = {res['fp8'] / res['bf16']:.3f} "
              f"(ring8 {os.environ.get('FT_DECODE_RING8', '2')}, wpc8 {os.environ.get('FT_DECODE_WPC8', '1')})", flush=True)


if __name__ == "__main__":
    main()
