"""fp8 decode attention: full kernel (ops.decode_attention on e4m3 caches) vs its bare
memory stream (bench/attn_fp8_diag.hip: same partition / ring at 4 waves per
workgroup, no math) with the kernel's V^T addressing (8 x 4-B loads per lane per
tile), with a fragment-ordered V layout (2 x 16-B loads), and K alone.  Cold caches
(KV copies alternate inside one hipGraph)."""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402
from gemm_sweep import graph_time  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libattnfp8diag.so"))
lib.attn8_loads_launch.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int] * 5 + \
    [ctypes.c_void_p, ctypes.c_void_p]
nq, nkv, d, bs = 32, 8, 128, 16
STREAMS = [(0, 2, "V^T b32 r2"), (1, 2, "V frag b128 r2"), (2, 2, "K only r2"), (0, 3, "V^T b32 r3"),
           (1, 3, "V frag b128 r3")]


def main():
    g = torch.Generator().manual_seed(0)
    sink = torch.zeros(256, dtype=torch.int32, device="cuda")
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
        kvs = [(torch.randn(total + 8, nkv, bs, d, device="cuda").to(torch.float8_e4m3fn),
                torch.randn(total + 8, nkv, d, bs, device="cuda").to(torch.float8_e4m3fn)) for _ in range(6)]
        nbytes = sum(lens) * nkv * d * 2
        full = graph_time([(lambda k=k, v=v: ops.decode_attention(out, q, k, v, bt, sl, tmp[0], tmp[1], nq, nkv, d,
                                                                  d ** -0.5, counters=cnt)) for k, v in kvs] * 4)
        res = [f"B={B} ctx {lo}-{hi} {nbytes / 1e6:.0f} MB: full {full:6.1f} us ({nbytes / full / 1e6:.2f} TB/s)"]
        for mode, ring, name in STREAMS:
            def call(kv, mode=mode, ring=ring):
                return lambda: lib.attn8_loads_launch(kv[0].data_ptr(), kv[1].data_ptr(), bt.data_ptr(),
                                                      bt.stride(0), sl.data_ptr(), B, nkv, mode, ring,
                                                      bs.bit_length() - 1, sink.data_ptr(),
                                                      torch.cuda.current_stream().cuda_stream)
            assert call(kvs[0])() == 0
            t = graph_time([call(kv) for kv in kvs] * 4)
            frac = 0.5 if mode == 2 else 1.0
            res.append(f"{name} {t:6.1f} ({frac * nbytes / t / 1e6:.2f} TB/s)")
        print("  ".join(res), flush=True)
        del kvs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
