"""Mixed prefill+decode step anatomy at the driver config's turn boundary: D
sequences keep decoding on ~CTX-token histories while P new turns (a cached
CTX-token history + NEW fresh tokens each) are prefilled in the same step --
what every bench turn starts with (step trace: ~34 decode rows + ~750 prefill
tokens, profiles/step_trace_driver_config_r02.txt).

Reports per mixed step: host time before the first kernel (schedule + input
build + upload), the enqueue time of the forward, GPU time (events), wall.

python bench/mixed_probe.py [--decode 34] [--new 7] [--ctx 3000] [--fresh 107] [--reps 6]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--decode", type=int, default=34)
    ap.add_argument("--new", type=int, default=7)
    ap.add_argument("--ctx", type=int, default=3000)
    ap.add_argument("--fresh", type=int, default=107)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--prof", action="store_true", help="torch.profiler kernel table of the mixed steps")
    a = ap.parse_args()

    import numpy as np
    import torch

    from fasttalk_llm_microservice_amd.engine.config import EngineConfig
    from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams

    eng = LLMEngine(EngineConfig(model=a.model, max_num_seqs=256))
    eng.runner.warmup([b for b in eng.runner.graph_sizes if b <= 64])
    rng = np.random.default_rng(0)
    sp = SamplingParams(temperature=0.7, top_p=0.9, max_tokens=4000, ignore_eos=True)
    hist = [rng.integers(0, 120000, a.ctx).tolist() for _ in range(a.decode + a.new * (a.reps + 1))]
    for i in range(a.decode):
        eng.add_request(f"d{i}", hist[i], sp)
    # warm the prefix cache with the histories of the turns to come
    for i in range(a.decode, len(hist)):
        eng.add_request(f"w{i}", hist[i], SamplingParams(temperature=0.0, max_tokens=1))
    while eng.scheduler.waiting or any(r.startswith("w") for r in eng.scheduler.by_id):
        eng.step()
    for _ in range(3):
        eng.step()
    r = eng.runner
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    rows = []
    orig_execute = r.execute

    def timed_execute(batch, masks):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record()
        out = orig_execute(batch, masks)
        ev1.record()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rows.append((len(batch.decode_seqs), sum(batch.prefill_tokens), 1e3 * (t1 - t0),
                     ev0.elapsed_time(ev1)))
        return out

    r.execute = timed_execute
    k = a.decode
    for rep in range(a.reps):
        for j in range(a.new):
            h = hist[k]
            k += 1
            eng.add_request(f"n{rep}_{j}", h + rng.integers(0, 120000, a.fresh).tolist(), sp)
        while eng._inflight:   # collect the queued decode steps: the next step is the mixed one
            eng.step()
        rows.clear()
        t0 = time.perf_counter()
        if a.prof and rep == a.reps - 1:
            from torch.profiler import ProfilerActivity, profile

            with profile(activities=[ProfilerActivity.CUDA]) as prof:
                eng.step()
                torch.cuda.synchronize()
            print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25, max_name_column_width=70))
        else:
            eng.step()
        wall = 1e3 * (time.perf_counter() - t0)
        nd, npf, ex_ms, gpu_ms = rows[0] if rows else (0, 0, 0, 0)
        print(f"mixed step: decode rows {nd} prefill tokens {npf}: wall {wall:.2f} ms, "
              f"execute {ex_ms:.2f} ms, GPU {gpu_ms:.2f} ms", flush=True)
        for j in range(a.new):
            eng.abort(f"n{rep}_{j}")
        for _ in range(2):
            eng.step()
    r.execute = orig_execute
    print("host profile", {k2: round(v, 4) for k2, v in eng.host_prof.items()})


if __name__ == "__main__":
    main()
