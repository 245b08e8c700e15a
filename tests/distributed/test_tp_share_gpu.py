"""A full TP=2 engine on ONE MI355X (VERDICT r1 "harden TP"): rank 0 is this
test process, rank 1 a spawned worker, both on cuda:0 (``tp_share_device``:
gloo for control -- RCCL refuses two ranks on one device -- and the custom
IPC all-reduce / all-gather for the data path, so decode steps replay hipGraphs
that contain the cross-process collectives).

* tokens match TP=1 of the same weights (``FT_CONSISTENT_INIT=1``: both draw
  the unsharded tensors from one host seed and slice them);
* fault contract: the worker stalls before one decode step until rank 0's
  all-reduce has run out of spin budget.  That step must FAIL (CommFault), never
  emit tokens computed from partial sums; the group switches to the fallback
  collectives on both ranks and the next requests reproduce the healthy run.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    from fasttalk_llm_microservice_amd.engine.config import EngineConfig

    # no prefix cache: repeated generations of the same prompts must recompute the
    # same way (greedy on random weights turns any rounding difference into new tokens)
    base = dict(model="tiny-2k", device="cuda", num_kv_blocks=512, max_model_len=1024,
                max_num_seqs=8, max_num_batched_tokens=256, graph_batch_sizes=(1, 2, 4, 8),
                enable_prefix_caching=False)
    base.update(kw)
    return EngineConfig(**base)


def _prompts():
    rng = np.random.default_rng(11)
    return [rng.integers(0, 120000, n).tolist() for n in (9, 40, 23)]


@pytest.fixture(scope="module")
def tp1_tokens():
    import torch

    from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams

    os.environ["FT_CONSISTENT_INIT"] = "1"
    sp = SamplingParams(temperature=0, max_tokens=12, ignore_eos=True)
    eng = LLMEngine(_cfg())
    out = eng.generate(_prompts(), sp)
    del eng
    torch.cuda.empty_cache()
    return out


def _agree(a, b):
    same = sum(x == y for p, q in zip(a, b) for x, y in zip(p, q))
    return same / sum(len(p) for p in a)


def _common_prefix(a, b):
    """Shortest run of leading tokens the two generations share, over the prompts:
    bf16 TP=2 and TP=1 round differently, and greedy decoding on random weights
    turns the first flipped near-tie into a different continuation."""
    out = []
    for p, q in zip(a, b):
        n = 0
        while n < min(len(p), len(q)) and p[n] == q[n]:
            n += 1
        out.append(n)
    return min(out)


def test_tp2_on_one_gpu_matches_tp1_and_survives_an_allreduce_timeout(tp1_tokens, monkeypatch):
    from fasttalk_llm_microservice_amd.engine.runner import CommFault
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
    from fasttalk_llm_microservice_amd.parallel.tp import spawn_tp_engine

    monkeypatch.setenv("FT_CONSISTENT_INIT", "1")
    # the worker's 20th decode-graph message (inside the second generation below)
    # stalls until rank 0's all-reduce has timed out (<= 60 s)
    monkeypatch.setenv("FT_FAULT_TP_STALL", "20:60")
    monkeypatch.setenv("ENGINE_CUSTOM_AR_SPIN", str(1 << 20))
    monkeypatch.setenv("ENGINE_TP_WARM_STEPS", "0")
    eng = spawn_tp_engine(_cfg(tp_size=2, tp_share_device=True, custom_allreduce=True))
    try:
        r = eng.runner
        assert r.comm.custom is not None and r.use_graphs
        assert eng.tp_group.alive()
        sp = SamplingParams(temperature=0, max_tokens=12, ignore_eos=True)
        # --- healthy run: decode graphs with the custom collectives ---
        ref2 = eng.generate(_prompts(), sp)
        assert r.stats["graph_replays"] > 0 and not r.comm.custom.failed
        # --- the faulting run ---
        for i, p in enumerate(_prompts()):
            eng.add_request(f"f{i}", p, sp)
        emitted, fault = {}, None
        for _ in range(200):
            if not eng.has_work():
                break
            try:
                for o in eng.step():
                    emitted.setdefault(o.request_id, []).extend(o.token_ids)
            except CommFault as e:
                fault = e
                eng.fail_unfinished(str(e))
                break
        assert fault is not None, "the stalled worker must make rank 0's all-reduce time out"
        assert r.comm.custom.failed and not r.graphs
        # tokens emitted before the fault are prefixes of the healthy run's: nothing
        # computed from partial sums reached a stream
        for i, ref in enumerate(ref2):
            got = emitted.get(f"f{i}", [])
            assert got == ref[:len(got)], (i, got, ref)
        # --- after the fallback (gloo host staging, eager): the healthy run again ---
        out = eng.generate(_prompts(), sp)
        assert eng.tp_group.alive()
    finally:
        eng.shutdown()
    print("post-fallback vs healthy TP2:", _agree(out, ref2), " TP2 vs TP1:", _agree(ref2, tp1_tokens))
    assert out == ref2          # same kernels, the fallback sums the same two fp32 values
    # greedy tokens of random weights: the first (prefill) token must agree; later ones
    # drift at near-ties (TP=2 sums two fp32 partials); the numerics check is on logits
    # (test_tp2_on_one_gpu_teacher_forced_logits_match_tp1)
    assert _common_prefix(ref2, tp1_tokens) >= 1


def test_tp2_on_one_gpu_graph_decode_matches_tp1(tp1_tokens, monkeypatch):
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
    from fasttalk_llm_microservice_amd.parallel.tp import spawn_tp_engine

    monkeypatch.setenv("FT_CONSISTENT_INIT", "1")
    monkeypatch.delenv("FT_FAULT_TP_STALL", raising=False)
    eng = spawn_tp_engine(_cfg(tp_size=2, tp_share_device=True, custom_allreduce=True))
    try:
        sp = SamplingParams(temperature=0, max_tokens=12, ignore_eos=True)
        out = eng.generate(_prompts(), sp)
        st = eng.runner.stats
        healthy = eng.runner.comm.custom.healthy()
    finally:
        eng.shutdown()
    assert healthy and st["graph_replays"] > 0, st
    print("TP2 vs TP1 token agreement", _agree(out, tp1_tokens), "common prefix",
          _common_prefix(out, tp1_tokens))
    assert _common_prefix(out, tp1_tokens) >= 1, (out, tp1_tokens)


def _teacher_forced_logits(eng, seqs):
    """Logits of one prefill step per sequence (max_tokens=1): row i predicts the token
    after seqs[i].  Eager steps only (the runner's logits tap)."""
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams

    sp = SamplingParams(temperature=0, max_tokens=1, ignore_eos=True)
    rows = []
    for q in seqs:
        eng.runner.logits_tap = []
        eng.generate([q], sp)
        rows.append(eng.runner.logits_tap[-1][-1])
        eng.runner.logits_tap = None
    import torch

    return torch.stack(rows)


def test_tp2_on_one_gpu_teacher_forced_logits_match_tp1(tp1_tokens, monkeypatch):
    """TP=2 (custom all-reduce + all-gather, both ranks on one MI355X) against TP=1 on
    the same weights, compared where it is well defined: the logits of the same
    inputs.  Each prompt is extended by the first k tokens of TP=1's greedy
    continuation (teacher forcing, k = 0..5), so the prefill GEMMs, the varlen
    attention over the paged cache and both collectives are all exercised; greedy
    tokens alone flip at random-weight near-ties."""
    import torch

    from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
    from fasttalk_llm_microservice_amd.parallel.tp import spawn_tp_engine

    monkeypatch.setenv("FT_CONSISTENT_INIT", "1")
    monkeypatch.delenv("FT_FAULT_TP_STALL", raising=False)
    seqs = [p + c[:k] for p, c in zip(_prompts(), tp1_tokens) for k in range(6)]
    eng1 = LLMEngine(_cfg())
    ref = _teacher_forced_logits(eng1, seqs)
    del eng1
    torch.cuda.empty_cache()
    eng = spawn_tp_engine(_cfg(tp_size=2, tp_share_device=True, custom_allreduce=True))
    try:
        assert eng.runner.comm.custom is not None
        got = _teacher_forced_logits(eng, seqs)
        healthy = eng.runner.comm.custom.healthy()
    finally:
        eng.shutdown()
    assert healthy and got.shape == ref.shape
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    agree = (got.argmax(-1) == ref.argmax(-1)).float().mean().item()
    print(f"TP2 vs TP1 teacher-forced logits: min cos {cos.min().item():.6f}, argmax agree {agree:.3f}")
    assert cos.min().item() > 0.999, cos
    assert agree >= 0.75


def test_tp2_allreduce_timeout_in_a_no_logits_prefill_chunk(monkeypatch):
    """a middle chunk of a chunked prefill samples nothing; a custom
    all-reduce timeout there must fail THAT step (before post_step commits its
    KV blocks to the prefix cache), and a CommFault empties the prefix cache."""
    from fasttalk_llm_microservice_amd.engine.runner import CommFault
    from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
    from fasttalk_llm_microservice_amd.parallel.tp import spawn_tp_engine

    monkeypatch.setenv("FT_CONSISTENT_INIT", "1")
    monkeypatch.setenv("FT_FAULT_TP_STALL", "m1:60")   # the worker's first eager step
    monkeypatch.setenv("ENGINE_CUSTOM_AR_SPIN", str(1 << 20))
    monkeypatch.setenv("ENGINE_TP_WARM_STEPS", "0")    # no long first-step waits
    eng = spawn_tp_engine(_cfg(tp_size=2, tp_share_device=True, custom_allreduce=True,
                               enable_prefix_caching=True, max_num_batched_tokens=64))
    try:
        rng = np.random.default_rng(5)
        prompt = rng.integers(0, 120000, 200).tolist()       # 4 chunks of 64 tokens
        sp = SamplingParams(temperature=0, max_tokens=4, ignore_eos=True)
        eng.add_request("p0", prompt, sp)
        fault = None
        for _ in range(20):
            try:
                eng.step()
            except CommFault as e:
                fault = e
                break
        assert fault is not None, "the stalled chunk must fail its own step"
        # the failing step was the first (no-logits) chunk: nothing was committed
        assert eng.runner.stats["prefill_steps"] == 1
        eng.fail_unfinished(str(fault), reset_cache=True)
        assert eng.bm.num_cached() == 0 and eng.bm.num_free() == eng.bm.num_blocks
        out = eng.generate([prompt], sp)                    # fallback collectives
        assert len(out[0]) == 4 and eng.tp_group.alive()
    finally:
        eng.shutdown()
