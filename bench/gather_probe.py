"""Host cost of the mixed step's id gather while the GPU is busy (is any form
synchronous?): index_select(out=), index_copy_, advanced indexing."""
import time

import torch

dev = "cuda"
d_out = torch.randint(0, 1000, (256,), dtype=torch.int32, device=dev)
buf = torch.zeros(4096, dtype=torch.int32, device=dev)
idx = torch.arange(50, dtype=torch.int64, device=dev)
dst = torch.arange(50, dtype=torch.int64, device=dev)
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)


def busy():
    for _ in range(20):
        a @ a   # ~ms of queued GPU work


forms = {
    "index_select_out": lambda: torch.index_select(d_out, 0, idx, out=buf[16:66]),
    "index_select_new": lambda: d_out.index_select(0, idx),
    "index_copy": lambda: buf[16:66].index_copy_(0, dst, d_out.index_select(0, idx)),
    "adv_index_copy": lambda: buf[16:66].copy_(d_out[idx]),
    "take": lambda: buf[16:66].copy_(torch.take(d_out, idx)),
}
for name, f in forms.items():
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        busy()
        t0 = time.perf_counter()
        f()
        ts.append(1e3 * (time.perf_counter() - t0))
        torch.cuda.synchronize()
    print(f"{name:20s} host ms: min {min(ts):.3f} median {sorted(ts)[5]:.3f} max {max(ts):.3f}", flush=True)
