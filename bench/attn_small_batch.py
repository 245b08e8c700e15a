"""Decode attention at small batches (single / few sessions, 3k-token histories):
in-launch combine (counters) vs the separate combine kernel, under the
process's FT_DECODE_* knobs.  Prints us per call for B = 1, 2, 4, 8, 16.

python bench/attn_small_batch.py            (one config per process: knobs read once)
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402
from gemm_sweep import graph_time  # noqa: E402


def main():
    nq, nkv, d, bs, ctx = 32, 8, 128, 16, 3000
    torch.manual_seed(0)
    res = []
    for B in (1, 2, 4, 8, 16):
        nblk = math.ceil(ctx / bs)
        nblocks = B * nblk + 8
        kvs = [(torch.randn(nblocks, nkv, bs, d, device="cuda").bfloat16(),
                torch.randn(nblocks, nkv, d, bs, device="cuda").bfloat16()) for _ in range(2)]
        bt = torch.randperm(nblocks, device="cuda")[: B * nblk].int().view(B, nblk)
        sl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        q = torch.randn(B, (nq + 2 * nkv) * d, device="cuda").bfloat16()
        outs = {}
        for fc in (True, False):
            out = torch.empty(B, nq * d, device="cuda").bfloat16()
            n_out, n_ml = ops.decode_workspace(B, nq, nkv, d)
            to, tm = torch.empty(n_out, device="cuda"), torch.empty(n_ml, device="cuda")
            cnt = ops.decode_counters(B, nkv, "cuda") if fc else None
            t = graph_time([lambda kv=kvs[i % 2]: ops.decode_attention(out, q, kv[0], kv[1], bt, sl, to, tm, nq,
                                                                       nkv, d, d ** -0.5, counters=cnt)
                            for i in range(8)])
            outs[fc] = (t, out.float())
        err = (outs[True][1] - outs[False][1]).abs().max().item()
        res.append(f"B={B}: fc {outs[True][0]:5.1f} us  sep {outs[False][0]:5.1f} us  (max diff {err:.1e})")
        del kvs
    print(" | ".join(res), flush=True)


if __name__ == "__main__":
    main()
