"""HBM streaming ceiling at decode-GEMM sizes: cold-cache read bandwidth of a
plain device copy (bytes read + written) and of a reduction (read only), for
the per-layer weight sizes of Llama-3-8B.  Captured in a hipGraph so launch
overhead is excluded; every call touches a different buffer (> MALL)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gemm_sweep import graph_time  # noqa: E402

for name, nbytes in [("o 33.5MB", 4096 * 4096 * 2), ("qkv 50MB", 6144 * 4096 * 2),
                     ("down 117MB", 4096 * 14336 * 2), ("gate_up 235MB", 28672 * 4096 * 2)]:
    n = nbytes // 2
    ncopy = max(2, min(24, (768 << 20) // nbytes))
    srcs = [torch.randn(n, device="cuda").bfloat16() for _ in range(ncopy)]
    dst = torch.empty(n, device="cuda").bfloat16()
    red = torch.empty(1, device="cuda")
    calls = 24
    t_copy = graph_time([lambda s=srcs[i % ncopy]: dst.copy_(s) for i in range(calls)])
    t_sum = graph_time([lambda s=srcs[i % ncopy]: torch.sum(s.view(-1, 4096), dim=0, out=None)
                        for i in range(calls)])
    print(f"{name:14s} copy {t_copy:7.2f} us ({2 * nbytes / t_copy / 1e3:5.0f} GB/s r+w)   "
          f"colsum {t_sum:7.2f} us ({nbytes / t_sum / 1e3:5.0f} GB/s read)", flush=True)
    del srcs
    torch.cuda.empty_cache()
