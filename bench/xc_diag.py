"""Splits the xc decode GEMM's time at 50 rows into its parts (bench/xc_diag.hip):
full / no slab stores / weight loads only / loads + x staging, cold cache, in a
hipGraph, next to the streaming-read ceiling of the same bytes (bench/bw_read.py)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402
from gemm_sweep import graph_time  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libxcdiag.so"))
lib.xc_diag_launch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
M = int(os.environ.get("ROWS", "50"))
for name, n, k, splits in [("o", 4096, 4096, 8), ("o", 4096, 4096, 4), ("qkv", 6144, 4096, 8),
                           ("qkv", 6144, 4096, 4), ("down", 4096, 14336, 4), ("down", 4096, 14336, 7),
                           ("gu", 28672, 4096, 2), ("gu", 28672, 4096, 1)]:
    if k % (512 * splits):
        continue
    copies = max(2, -(-(768 << 20) // (n * k * 2)))
    ws_ = [ops.pack_weight(torch.randn(n, k, device="cuda").bfloat16()) for _ in range(copies)]
    x = torch.randn(M, k, device="cuda").bfloat16()
    slab = torch.empty(splits * M * n, device="cuda")
    row = []
    for d in range(4):
        def call(w, d=d):
            return lambda: lib.xc_diag_launch(x.data_ptr(), M, w.data_ptr(), n, k, slab.data_ptr(), splits, d,
                                              torch.cuda.current_stream().cuda_stream)
        assert call(ws_[0])() == 0
        row.append(graph_time([call(ws_[i % copies]) for i in range(max(copies, 8))]))
    print(f"{name:5s} n={n:5d} k={k:5d} split {splits}: full {row[0]:6.2f}  no-store {row[1]:6.2f}  "
          f"loads {row[2]:6.2f}  loads+x {row[3]:6.2f} us  ({n * k * 2 / row[0] / 1e3:.0f} GB/s full)", flush=True)
    del ws_
    torch.cuda.empty_cache()
