"""Decode attention: full kernel (ops.decode_attention, incl. combine) vs its bare
memory stream (bench/attn_diag.hip: same partition / addressing / ring, no math)
vs the streaming-read ceiling of the same bytes.  Two KV copies alternate so
every call reads cold."""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402
from gemm_sweep import graph_time  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libattndiag.so"))
lib.attn_loads_launch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 6 + \
    [ctypes.c_void_p, ctypes.c_void_p]
nq, nkv, d = 32, 8, 128
bs = int(os.environ.get("BS", "16"))   # KV block size (tokens)
STREAMS = [(0, 3, 2, "K+V r3"), (4, 3, 2, "K+V nt r3"), (4, 4, 2, "K+V nt r4"), (3, 3, 2, "contig r3")]
if os.environ.get("SWEEP"):  # ring x workgroups-per-CU of the nt stream
    STREAMS = [(4, r, w, f"nt r{r} w{w}") for r in (2, 3, 4) for w in (1, 2, 3, 4)]
sink = torch.zeros(256, dtype=torch.int32, device="cuda")
for B, ctx, uniform in [(50, 3000, False), (50, 4500, False), (64, 4096, True)]:
    nblk = math.ceil(ctx / bs)
    nblocks = B * nblk + 8
    kvs = [(torch.randn(nblocks, nkv, bs, d, device="cuda").bfloat16(),
            torch.randn(nblocks, nkv, d, bs, device="cuda").bfloat16()) for _ in range(2)]
    order = os.environ.get("ORDER", "rand")
    if order == "seq":      # each sequence's blocks contiguous
        bt = torch.arange(B * nblk, device="cuda").int().view(B, nblk)
    elif order == "chunk":  # runs of 64 contiguous blocks (1 MiB per kv head), run order shuffled
        runs = torch.randperm(B * nblk // 64, device="cuda")
        bt = (runs[:, None] * 64 + torch.arange(64, device="cuda")[None]).flatten()
        bt = torch.cat([bt, torch.arange(bt.numel(), B * nblk, device="cuda")]).int().view(B, nblk)
    else:
        bt = torch.randperm(nblocks, device="cuda")[: B * nblk].int().view(B, nblk)
    print("block order", order, "bs", bs, flush=True) if B == 50 and ctx == 3000 else None
    sl = torch.full((B,), ctx, dtype=torch.int32, device="cuda") if uniform else \
        torch.randint(ctx // 2, ctx + 1, (B,), dtype=torch.int32, device="cuda")
    q = torch.randn(B, (nq + 2 * nkv) * d, device="cuda").bfloat16()
    out = torch.empty(B, nq * d, device="cuda").bfloat16()
    n_out, n_ml = ops.decode_workspace(B, nq, nkv, d)
    to, tm = torch.empty(n_out, device="cuda"), torch.empty(n_ml, device="cuda")
    nbytes = int(sl.sum().item()) * nkv * d * 4
    full = graph_time([lambda kv=kvs[i % 2]: ops.decode_attention(out, q, kv[0], kv[1], bt, sl, to, tm, nq, nkv, d,
                                                                  d ** -0.5) for i in range(8)])
    cnt = ops.decode_counters(B, nkv, "cuda")
    fused = graph_time([lambda kv=kvs[i % 2]: ops.decode_attention(out, q, kv[0], kv[1], bt, sl, to, tm, nq, nkv,
                                                                   d, d ** -0.5, counters=cnt) for i in range(8)])
    res = [f"B={B} ctx={ctx}{' uniform' if uniform else ''} {nbytes / 1e6:.0f} MB: full {full:7.1f} us "
           f"({nbytes / full / 1e3:.0f} GB/s) fused-combine {fused:7.1f}"]
    for mode, ring, wpc, name in STREAMS:
        def call(kv, mode=mode, ring=ring, wpc=wpc):
            return lambda: lib.attn_loads_launch(kv[0].data_ptr(), kv[1].data_ptr(), bt.data_ptr(), bt.stride(0),
                                                 sl.data_ptr(), B, nkv, mode, ring, wpc, bs.bit_length() - 1,
                                                 sink.data_ptr(),
                                                 torch.cuda.current_stream().cuda_stream)
        assert call(kvs[0])() == 0
        t = graph_time([call(kvs[i % 2]) for i in range(8)])
        frac = 0.5 if mode in (1, 2) else 1.0
        res.append(f"{name} {t:6.1f} ({frac * nbytes / t / 1e3:.0f} GB/s)")
    print("  ".join(res), flush=True)
    del kvs
    torch.cuda.empty_cache()
