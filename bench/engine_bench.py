"""Engine-level throughput probe (no WebSocket): N concurrent sequences through
LLMEngine.step(), reports decode tok/s, step latency and the runner stats.

python bench/engine_bench.py --model llama3.1-8b --seqs 50 --prompt 512 --gen 256
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3.1-8b")
    ap.add_argument("--seqs", type=int, default=50)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--gen", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--temperature", type=float, default=0.7)
    ap.add_argument("--kv-blocks", type=int, default=None)
    ap.add_argument("--batch-invariant", action="store_true")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"])
    a = ap.parse_args()

    import numpy as np
    import torch

    from fasttalk_llm_microservice_amd.engine.config import EngineConfig
    from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams

    cfg = EngineConfig(model=a.model, enforce_eager=a.eager, num_kv_blocks=a.kv_blocks,
                       batch_invariant=a.batch_invariant, kv_cache_dtype=a.kv_cache_dtype)
    t0 = time.time()
    eng = LLMEngine(cfg)
    print(f"engine up in {time.time() - t0:.1f}s", flush=True)
    rng = np.random.default_rng(0)
    res = []
    for r in range(a.rounds):
        prompts = [rng.integers(0, 120000, a.prompt).tolist() for _ in range(a.seqs)]
        sp = SamplingParams(temperature=a.temperature, top_p=0.9, max_tokens=a.gen, ignore_eos=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i, p in enumerate(prompts):
            eng.add_request(f"r{r}-{i}", p, SamplingParams(**sp.__dict__))
        first = None
        ntok = 0
        while eng.has_work():
            outs = eng.step()
            ntok += sum(len(o.token_ids) for o in outs)
            if first is None and outs:
                first = time.perf_counter() - t0
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        m = eng.metrics()
        res.append({"round": r, "tokens": ntok, "seconds": dt, "tok_s": ntok / dt,
                    "ttft_s": first, "decode_step_ms": m["decode_step_ms_avg"],
                    "prefill_step_ms": m["prefill_step_ms_avg"]})
        print(json.dumps(res[-1]), flush=True)
    print(json.dumps({"final": res[-1], "runner": eng.runner.stats}), flush=True)


if __name__ == "__main__":
    main()
