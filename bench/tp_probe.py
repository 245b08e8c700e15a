"""TP decode step on ONE MI355X (both ranks share the device, ENGINE_TP_SHARE_DEVICE:
gloo control + the custom IPC collectives, decode graphs replayed): a 2-layer
Llama-3-70B-shaped model (H 8192, I 28672, 64 q / 8 kv heads), TP=2, 50 sessions
on ~CTX-token histories.  Reports the engine's decode step with the fused
all-reduce + add + RMSNorm epilogue (FT_TP_FUSED_NORM=1, default) or the
separate slab_store -> all-reduce -> add+RMSNorm launches (=0).  Both ranks' kernels
run on the same GPU, so a step costs about twice a real TP=2 step; the A/B
difference is the launches saved.  Kernel counts per step: run under rocprofv3.

python bench/tp_probe.py [--sessions 50] [--ctx 2000] [--steps 40]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b-2l")
    ap.add_argument("--sessions", type=int, default=50)
    ap.add_argument("--ctx", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--tp", type=int, default=2)
    a = ap.parse_args()
    import numpy as np
    import torch

    from fasttalk_llm_microservice_amd.engine.config import EngineConfig
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
    from fasttalk_llm_microservice_amd.parallel.tp import spawn_tp_engine

    cfg = EngineConfig(model=a.model, device="cuda", tp_size=a.tp, tp_share_device=True,
                       custom_allreduce=True, max_model_len=8192, max_num_seqs=64,
                       num_kv_blocks=(a.sessions * (a.ctx + a.steps + 64)) // 16 + 64,
                       graph_batch_sizes=(a.sessions,), gpu_memory_utilization=0.4)
    eng = spawn_tp_engine(cfg)
    try:
        r = eng.runner
        rng = np.random.default_rng(0)
        sp = SamplingParams(temperature=0.0, max_tokens=a.steps + 40, ignore_eos=True)
        for i in range(a.sessions):
            eng.add_request(f"s{i}", rng.integers(0, 120000, a.ctx).tolist(), sp)
        while eng.scheduler.waiting:
            eng.step()
        for _ in range(5):
            eng.step()
        torch.cuda.synchronize()
        n0 = eng.stats["decode_steps"]
        t0 = time.perf_counter()
        for _ in range(a.steps):
            eng.step()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        n = eng.stats["decode_steps"] - n0
        print(f"{a.model} TP={a.tp} (ranks share one GPU) {a.sessions} sessions ctx {a.ctx}: "
              f"decode step {1e3 * dt / max(n, 1):.3f} ms over {n} steps "
              f"(fused AR+norm {'on' if r.model.tp_fused_norm else 'off'}, "
              f"custom collectives {'on' if r.comm.custom is not None and not r.comm.custom.failed else 'off'}, "
              f"graph replays {r.stats['graph_replays']})", flush=True)
    finally:
        eng.shutdown()


if __name__ == "__main__":
    main()
