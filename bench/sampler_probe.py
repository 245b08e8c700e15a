"""Sampler kernel timing at the serving shape ([rows, 128256] bf16 logits) per
mode: greedy / temperature / top-p / top-k (+top-p); hipGraph of 100 calls, each on its own
decode step (fresh uniforms, as in serving: top-p rows whose candidates are all rejected -- the
slow one-workgroup tail -- show up at their real rate).

python bench/sampler_probe.py [--rows 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from fasttalk_llm_microservice_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50)
    a = ap.parse_args()
    b, v, dev = a.rows, 128256, "cuda"
    logits = (torch.randn(b, v, device=dev) * 2).bfloat16()
    seeds = torch.arange(b, dtype=torch.int64, device=dev)
    n_calls = 100
    steps = torch.arange(n_calls, dtype=torch.int32, device=dev)[:, None].repeat(1, b).contiguous()
    for name, t, p, k in (("greedy", 0.0, 1.0, 0), ("temp", 0.7, 1.0, 0), ("top_p", 0.7, 0.9, 0),
                          ("top_k", 0.7, 1.0, 40), ("top_k+top_p", 0.7, 0.9, 40)):
        tt = torch.full((b,), t, device=dev)
        pp = torch.full((b,), p, device=dev)
        kk = torch.full((b,), k, dtype=torch.int32, device=dev)
        ops.sample(logits, tt, pp, kk, seeds, steps[0])
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(n_calls):
                ops.sample(logits, tt, pp, kk, seeds, steps[i])
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(2):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:12s} rows={b}: {e0.elapsed_time(e1) * 1e3 / (2 * n_calls):7.2f} us", flush=True)


if __name__ == "__main__":
    main()
