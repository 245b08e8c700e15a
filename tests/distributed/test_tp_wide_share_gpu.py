"""Tensor parallelism at W = 4 and 8 with every rank on ONE MI355X (VERDICT r3
"Next round" #1: BASELINE config 4, Llama-3-70B TP=8, had never executed).

Rank 0 is this test process, ranks 1..W-1 are spawned workers, all on cuda:0
(``tp_share_device``: gloo for control, the custom IPC all-reduce / fused
all-reduce + add + RMSNorm / logits all-gather for the data path), so the W=4 /
W=8 kernel instances, the shm step ring with W-1 readers and the lock-step
decode-graph capture across W processes all run.

Numerics are checked where they are well defined -- logits of the same inputs --
for EVERY step of a greedy generation: the eager prefill step and each
graph-replayed decode step of the TP=W engine are compared against TP=1 of the
same weights (``FT_CONSISTENT_INIT``) fed the same tokens (the TP=W engine's own
greedy continuation, teacher-forced through TP=1 prefill steps).

Shapes: ``tiny-2k`` (16 q / 4 kv heads of d=128: W=8 replicates each kv head on
two ranks) and ``llama3-70b-2l`` at W=8, the per-rank shapes of config 4
(qkv 1280, o 1024 -> 8192, gate_up 7168, down 3584 -> 8192, LM head 16032 rows).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cfg(model, **kw):
    from fasttalk_llm_microservice_amd.engine.config import EngineConfig

    base = dict(model=model, device="cuda", num_kv_blocks=256, max_model_len=1024,
                max_num_seqs=8, max_num_batched_tokens=256, graph_batch_sizes=(1, 2, 4, 8),
                enable_prefix_caching=False)
    base.update(kw)
    return EngineConfig(**base)


def _prompts():
    rng = np.random.default_rng(17)
    return [rng.integers(0, 120000, n).tolist() for n in (11, 37, 24)]


def _rows_by_request(tap, tap_ids):
    """{request id: [logits row of step 0, step 1, ...]} from the runner's tap."""
    out = {}
    for logits, ids in zip(tap, tap_ids):
        logits = logits.cpu()
        for i, rid in enumerate(ids or []):
            out.setdefault(rid, []).append(logits[i])
    return out


def _tp1_teacher_forced(model, seqs):
    import torch

    from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams

    eng = LLMEngine(_cfg(model))
    sp = SamplingParams(temperature=0, max_tokens=1, ignore_eos=True)
    rows = []
    for q in seqs:
        eng.runner.logits_tap = []
        eng.generate([q], sp)
        rows.append(eng.runner.logits_tap[-1][-1])
    eng.runner.logits_tap = None
    del eng
    torch.cuda.empty_cache()
    return torch.stack(rows)


@pytest.mark.parametrize("tp,model", [(4, "tiny-2k"), (8, "tiny-2k"), (4, "llama3-70b-2l"),
                                      (8, "llama3-70b-2l")])
def test_tp_wide_one_gpu_every_step_logits_match_tp1(tp, model, monkeypatch):
    import torch

    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
    from fasttalk_llm_microservice_amd.parallel.tp import spawn_tp_engine

    monkeypatch.setenv("FT_CONSISTENT_INIT", "device")
    monkeypatch.delenv("FT_FAULT_TP_STALL", raising=False)
    steps = 8
    sp = SamplingParams(temperature=0, max_tokens=steps, ignore_eos=True)
    eng = spawn_tp_engine(_cfg(model, tp_size=tp, tp_share_device=True, custom_allreduce=True))
    try:
        r = eng.runner
        assert r.comm.custom is not None and r.comm.world_size == tp and r.use_graphs
        assert eng.tp_group.alive() and len(eng.tp_group.procs) == tp - 1
        r.logits_tap, r.logits_tap_ids = [], []
        rids = []
        for i, p in enumerate(_prompts()):
            rid = f"w{tp}-{i}"
            eng.add_request(rid, p, sp)
            rids.append(rid)
        toks = {rid: [] for rid in rids}
        for _ in range(200):
            if not eng.has_work():
                break
            for o in eng.step():
                toks[o.request_id].extend(o.token_ids)
        tap = _rows_by_request(r.logits_tap, r.logits_tap_ids)
        r.logits_tap = r.logits_tap_ids = None
        st = dict(r.stats)
        healthy = r.comm.custom.healthy()
        # a second batch with a different composition (graph bucket 1, then 2)
        again = eng.generate(_prompts()[:2], SamplingParams(temperature=0, max_tokens=4,
                                                            ignore_eos=True))
        alive = eng.tp_group.alive()
    finally:
        eng.shutdown()
    assert healthy and alive, "a custom collective timed out or a worker died"
    assert st["graph_replays"] >= steps - 1, st
    assert all(len(toks[rid]) == steps for rid in rids), toks
    assert all(len(a) == 4 for a in again)
    seqs, got = [], []
    for rid, p in zip(rids, _prompts()):
        # (a pipelined step queued past max_tokens may add a discarded row at the end)
        assert len(tap[rid]) >= steps, (rid, len(tap[rid]))
        for k in range(steps):      # step k predicted toks[k] from prompt + toks[:k]
            seqs.append(p + toks[rid][:k])
            got.append(tap[rid][k])
    got = torch.stack(got)
    ref = _tp1_teacher_forced(model, seqs)
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    agree = (got.argmax(-1) == ref.argmax(-1)).float().mean().item()
    print(f"TP{tp} {model} vs TP1, {len(seqs)} steps (prefill + graph decode): "
          f"min cos {cos.min().item():.6f}, argmax agree {agree:.3f}, stats {st}")
    assert cos.min().item() > 0.999, cos
    # decode steps (k >= 1) ran as hipGraph replays with the W-rank collectives inside
    assert cos.view(len(rids), steps)[:, 1:].min().item() > 0.999
    assert agree >= 0.75
