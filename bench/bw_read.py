"""HBM streaming-read ceiling at the decode sizes (weights of one projection,
one layer's KV at 50 x 3k): a plain read-only kernel (bench/bw_kernel.hip),
cold cache (buffers rotated through > 768 MiB), calls captured in one hipGraph.
Sweeps grid size, loads in flight per thread and access pattern, prints the
best GB/s per size: the bar the decode GEMMs and attention are measured against.

python bench/bw_read.py   (needs bench/libbwk.so: hipcc --offload-arch=gfx950 -O3 -shared -fPIC
                            bench/bw_kernel.hip -o bench/libbwk.so)
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gemm_sweep import graph_time  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libbwk.so"))
lib.bw_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                        ctypes.c_int, ctypes.c_void_p]
out = torch.empty(4096 * 256, dtype=torch.int32, device="cuda")

SIZES = [("o 33.5MB", 4096 * 4096 * 2), ("qkv 50MB", 6144 * 4096 * 2),
         ("down 117MB", 4096 * 14336 * 2), ("gate_up 235MB", 28672 * 4096 * 2),
         ("kv/layer 614MB", 50 * 3000 * 8 * 128 * 2 * 2)]
if os.environ.get("BW_SIZES_MB"):   # e.g. "8.4,16.8,66" (the W4 decode weight streams)
    SIZES = [(f"{v}MB", int(float(v) * (1 << 20)) // 4096 * 4096) for v in os.environ["BW_SIZES_MB"].split(",")]
BLOCKS = tuple(int(v) for v in os.environ.get("BW_BLOCKS", "256,512,1024,2048,4096").split(","))
for name, nbytes in SIZES:
    ncopy = max(2, min(24, (768 << 20) // nbytes + 1))
    bufs = [torch.empty(nbytes // 2, dtype=torch.bfloat16, device="cuda").normal_() for _ in range(ncopy)]
    best = (1e9, None)
    res = []
    for mode in (0, 1):
        for blocks in BLOCKS:
            for unroll in (2, 4, 8, 16):
                def call(b):
                    return lambda: lib.bw_read(b.data_ptr(), nbytes, out.data_ptr(), blocks, unroll, mode,
                                               torch.cuda.current_stream().cuda_stream)
                t = graph_time([call(bufs[i % ncopy]) for i in range(max(ncopy, 8))])
                res.append((t, mode, blocks, unroll))
                if t < best[0]:
                    best = (t, (mode, blocks, unroll))
    res.sort()
    if os.environ.get("BW_ALL"):
        for t, m, b, u in sorted(res, key=lambda r: (r[1], r[2], r[3])):
            print(f"  {name} mode {m} blocks {b:5d} unroll {u:2d}: {t:8.2f} us {nbytes / t / 1e3:6.0f} GB/s")
    print(f"{name:15s} best {best[0]:8.2f} us {nbytes / best[0] / 1e3:6.0f} GB/s  mode/blocks/unroll {best[1]}   "
          + "  ".join(f"{m}/{b}/{u}={t:.1f}" for t, m, b, u in res[1:6]), flush=True)
    del bufs
    torch.cuda.empty_cache()
