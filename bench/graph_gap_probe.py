"""Where does a pipelined decode step lose GPU time outside the kernels?

Builds the flagship engine (Llama-3-8B shape, random weights), prefills N
sequences of P tokens, then times the same decode step five ways:
  engine   LLMEngine.step() in the pipelined steady state (host fill + launch)
  replay   the captured decode graph replayed back to back (kernels only)
  +h2d     + the per-step pinned H2D input upload before each replay
  +ids     + the device-side copy of the sampled ids into the next step's input
  +d2h     + the D2H copy of the sampled ids and the event record (= the engine's
           _decode_enqueue minus the host fill)
python bench/graph_gap_probe.py --seqs 50 --prompt 3000
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
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seqs", type=int, default=50)
    ap.add_argument("--prompt", type=int, default=3000)
    ap.add_argument("--iters", type=int, default=60)
    a = ap.parse_args()

    import numpy as np
    import torch

    from fasttalk_llm_microservice_amd.engine.config import EngineConfig
    from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams

    eng = LLMEngine(EngineConfig(model=a.model, device="cuda"))
    rng = np.random.default_rng(0)
    for i in range(a.seqs):
        eng.add_request(f"r{i}", rng.integers(0, 120000, a.prompt).tolist(),
                        SamplingParams(temperature=0.7, top_p=0.9, max_tokens=4 * a.iters + 64,
                                       ignore_eos=True))
    while eng.stats["decode_steps"] < 8:
        eng.step()
    r = eng.runner
    torch.cuda.synchronize()
    out = {}
    t0 = time.perf_counter()
    for _ in range(a.iters):
        eng.step()
    torch.cuda.synchronize()
    out["engine"] = 1e3 * (time.perf_counter() - t0) / a.iters
    # drain the in-flight step, then drive the graph by hand
    while eng._inflight:
        eng.step()
    torch.cuda.synchronize()
    seqs = list(eng.scheduler.running)[: a.seqs]
    for s in seqs:  # the block for the next position (schedule() would allocate it)
        k = eng.scheduler._blocks_needed(s, s.n_tokens)
        if k:
            s.block_ids.extend(eng.bm.allocate(k))
    h = r.decode_launch(seqs)
    r.decode_collect(h)
    nb = r._bucket(len(seqs))
    g = r.graphs[nb]
    st = r.stg[0]
    nw = 10 * r.max_decode_batch + nb * r.max_blocks_per_seq

    def timed(body):
        body()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            body()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t) / a.iters

    def replay():
        g.replay()

    def h2d():
        r.d_in[:nw].copy_(st.h_in[:nw], non_blocking=True)
        g.replay()

    def ids():
        r.d_in[:nw].copy_(st.h_in[:nw], non_blocking=True)
        r.d_input_ids[:nb].copy_(r.d_out[:nb])
        g.replay()

    def d2h():
        r.d_in[:nw].copy_(st.h_in[:nw], non_blocking=True)
        r.d_input_ids[:nb].copy_(r.d_out[:nb])
        g.replay()
        st.h_out[:len(seqs)].copy_(r.d_out[:len(seqs)], non_blocking=True)
        st.event.record()

    for name, fn in (("replay", replay), ("+h2d", h2d), ("+ids", ids), ("+d2h", d2h)):
        out[name] = timed(fn)
    out = {k: round(v, 3) for k, v in out.items()}
    out.update(seqs=len(seqs), bucket=nb, prompt=a.prompt)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
