"""Does PyTorch TunableOp (exhaustive hipBLASLt/rocBLAS solution search) beat the
default heuristic at decode shapes?  Run with PYTORCH_TUNABLEOP_ENABLED=1."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch, torch.nn.functional as F
from kernel_bench import timeit
M = int(os.environ.get("M", "50"))
res = {}
for name, n, k in [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336), ("lm_head", 128256, 4096)]:
    W = (torch.randn(n, k, device="cuda") * 0.02).bfloat16()
    x = torch.randn(M, k, device="cuda").bfloat16()
    F.linear(x, W); torch.cuda.synchronize()
    t = timeit(lambda: F.linear(x, W), iters=100)
    res[name] = round(t, 2)
    print(name, f"{t:.2f}us {n*k*2/t/1e3:.0f}GB/s", flush=True)
print(json.dumps(res))
