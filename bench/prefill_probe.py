"""Prefill-attention probe at the multi-turn serving shape: S sequences each
prefilling a new chunk of Q tokens on top of a cached context of C tokens
(Llama-3-8B heads, scattered KV blocks).  Prints us/call, TFLOP/s and the KV
bytes/s the kernel streams.

python bench/prefill_probe.py [--cases 50:60:3000,8:512:0,1:2048:0]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402
from kernel_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="50:60:3000,50:60:1500,8:512:0,1:2048:0,4:1024:4096")
    ap.add_argument("--nq", type=int, default=32)
    ap.add_argument("--nkv", type=int, default=8)
    a = ap.parse_args()
    nq, nkv, d, bs = a.nq, a.nkv, 128, 16
    dev = "cuda"
    for case in a.cases.split(","):
        S, Q, C = (int(v) for v in case.split(":"))
        L = Q + C
        nblk = math.ceil(L / bs)
        nblocks = S * nblk + 8
        kc = torch.randn(nblocks, nkv, bs, d, device=dev).bfloat16()
        vc = torch.randn(nblocks, nkv, d, bs, device=dev).bfloat16()
        bt = torch.randperm(nblocks, device=dev)[: S * nblk].int().view(S, nblk)
        sl = torch.full((S,), L, dtype=torch.int32, device=dev)
        qsl = torch.arange(0, S * Q + 1, Q, dtype=torch.int32)
        T = S * Q
        q = torch.randn(T, nq * d, device=dev).bfloat16()
        tiles, comb = ops.build_prefill_tiles([Q] * S, ops.prefill_tile_tokens(nq, nkv),
                                              seq_lens=None if os.environ.get("NOSPLIT") else [L] * S,
                                              nkv=nkv)
        ti = torch.tensor(tiles, dtype=torch.int32, device=dev).flatten()
        n_po, n_pml = ops.prefill_partials(nkv, d)
        po, pml = torch.empty(n_po, device=dev), torch.empty(n_pml, device=dev)
        cb = torch.tensor(comb or [[0, 0, 0, 0]], dtype=torch.int32, device=dev).flatten()
        npart = sum(c[3] for c in comb)
        out = torch.empty(T, nq * d, device=dev).bfloat16()
        qd = qsl.to(dev)
        us = timeit(lambda: ops.prefill_attention(out, q, kc, vc, bt, sl, qd, ti, len(tiles), nq, nkv,
                                                  d, d ** -0.5, po, pml, cb, len(comb), npart),
                    iters=20, warmup=3)
        # causal FLOPs: each new token attends to C + its position in the chunk
        flops = 4 * d * nq * S * sum(C + i + 1 for i in range(Q))
        kv_bytes = S * L * nkv * d * 2 * 2
        print(json.dumps({"seqs": S, "new": Q, "ctx": C, "us": round(us, 1),
                          "TFLOPs": round(flops / us / 1e6, 1),
                          "KV_GBps": round(kv_bytes / us / 1e3, 1), "wgs": len(tiles) * nkv, "splits": npart}),
              flush=True)
        del kc, vc


if __name__ == "__main__":
    main()
