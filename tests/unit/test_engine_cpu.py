"""Engine tests on the CPU backend (no GPU): fp32 reference ops, scheduler
invariants with a fake runner (continuous batching, chunked prefill,
preemption, abort, stop handling), and the tiny random-init Llama end to end
(greedy determinism, chunked prefill == single shot, prefix cache does not
change outputs, guided JSON decoding)."""
import json
import math

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import EngineError, LLMEngine
from fasttalk_llm_microservice_amd.engine.guided import GuidedSpec
from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
from fasttalk_llm_microservice_amd.models.config import MODELS
from fasttalk_llm_microservice_amd.ops import reference as ref


# ----------------------------------------------------------------------------- reference ops
def test_reference_paged_attention_matches_dense():
    torch.manual_seed(0)
    nq, nkv, d, bs = 8, 2, 16, 4
    lens, qlens = [7, 13], [3, 13]
    nblk = sum(math.ceil(x / bs) for x in lens)
    kc = torch.randn(nblk, nkv, bs, d)
    vc = torch.randn(nblk, nkv, d, bs)   # V blocks transposed
    bt = torch.zeros(2, 4, dtype=torch.int32)
    bt[0, :2] = torch.tensor([3, 0])
    bt[1, :4] = torch.tensor([1, 2, 4, 5])
    q = torch.randn(sum(qlens), nq, d)
    qsl = torch.tensor([0, 3, 16], dtype=torch.int32)
    out = ref.paged_attention(q, kc, vc, bt, torch.tensor(lens), qsl, d ** -0.5)
    for b in range(2):
        k = ref._gather_kv(kc, bt[b], lens[b]).repeat_interleave(nq // nkv, 1)
        v = ref._gather_kv(vc, bt[b], lens[b], transposed=True).repeat_interleave(nq // nkv, 1)
        qq = q[qsl[b]:qsl[b + 1]].transpose(0, 1)
        L, ql = lens[b], qlens[b]
        mask = torch.ones(ql, L, dtype=torch.bool).tril(L - ql)
        o = torch.nn.functional.scaled_dot_product_attention(
            qq, k.transpose(0, 1), v.transpose(0, 1), attn_mask=mask, scale=d ** -0.5)
        torch.testing.assert_close(out[qsl[b]:qsl[b + 1]], o.transpose(0, 1), atol=1e-5, rtol=1e-5)


def test_reference_rope_and_kv_write():
    nq, nkv, d, bs = 4, 2, 8, 4
    cs = ref.rope_cos_sin(d, 64, 500000.0, {"rope_type": "llama3", "factor": 8.0,
                                            "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                            "original_max_position_embeddings": 8192})
    qkv = torch.randn(3, (nq + 2 * nkv) * d)
    orig = qkv.clone()
    kc = torch.zeros(4, nkv, bs, d)
    vc = torch.zeros(4, nkv, d, bs)
    pos = torch.tensor([0, 5, 9], dtype=torch.int32)
    slots = torch.tensor([1, 6, 13], dtype=torch.int32)
    ref.rope_kv_write(qkv, pos, cs, slots, kc, vc, nq, nkv, d)
    # position 0 leaves q unrotated; v is copied verbatim
    torch.testing.assert_close(qkv[0, : nq * d], orig[0, : nq * d])
    v_src = orig[2, (nq + nkv) * d:].view(nkv, d)
    torch.testing.assert_close(vc[13 // bs, :, :, 13 % bs], v_src)  # V blocks transposed
    # rotation preserves the norm of every head
    qn = qkv[1, : nq * d].view(nq, d).norm(dim=-1)
    torch.testing.assert_close(qn, orig[1, : nq * d].view(nq, d).norm(dim=-1))


def test_reference_sampler_contract():
    logits = torch.tensor([[0.0, 5.0, 1.0, 4.9], [3.0, 3.0, 0.0, 0.0]])
    z = torch.zeros(2)
    one = torch.ones(2)
    zi = torch.zeros(2, dtype=torch.int32)
    seeds = torch.tensor([1, 2])
    out = ref.sample(logits, z, one, zi, seeds, zi)
    assert out.tolist() == [1, 0]  # argmax, lowest id on ties
    # top_k = 1 is greedy whatever the temperature
    l2 = torch.tensor([[0.0, 5.0, 1.0, 4.9], [3.0, 2.5, 0.0, 0.0]])
    out = ref.sample(l2, one, one, torch.ones(2, dtype=torch.int32), seeds, zi)
    assert out.tolist() == [1, 0]
    # the allow-mask removes tokens
    mask = torch.tensor([[0b1000], [0b0100]], dtype=torch.int32)
    assert ref.sample(logits, z, one, zi, seeds, zi, mask=mask).tolist() == [3, 2]


# ----------------------------------------------------------------------------- fake runner
class FakeRunner:
    """Deterministic next token = (last token * 7 + 3) % 1000; records batches."""

    def __init__(self, num_blocks=64, max_model_len=512, eos_every=0):
        self.num_blocks = num_blocks
        self.max_model_len = max_model_len
        self.mcfg = MODELS["tiny"]
        self.dtype = torch.float32
        self.device = torch.device("cpu")
        self.stats = {"steps": 0}
        self.batches = []
        self.eos_every = eos_every

    def execute(self, batch, masks):
        self.stats["steps"] += 1
        self.batches.append((len(batch.decode_seqs), list(batch.prefill_tokens)))
        out = []
        for s in batch.sampled_seqs():
            nxt = (int(s.tokens[-1]) * 7 + 3) % 1000
            if self.eos_every and (s.n_tokens - s.prompt_len + 1) % self.eos_every == 0:
                nxt = 128009
            out.append(nxt)
        return out


def _fake_engine(**kw):
    runner_kw = {k: kw.pop(k) for k in list(kw) if k in ("num_blocks", "max_model_len", "eos_every")}
    cfg = EngineConfig(model="tiny", device="cpu", block_size=4, **kw)
    return LLMEngine(cfg, runner=FakeRunner(**runner_kw))


def _expected(prompt, n):
    out, last = [], prompt[-1]
    for _ in range(n):
        last = (last * 7 + 3) % 1000
        out.append(last)
    return out


def test_continuous_batching_and_chunked_prefill():
    eng = _fake_engine(max_num_seqs=8, max_num_batched_tokens=16)
    prompts = [list(range(1, 1 + n)) for n in (5, 40, 3, 17)]
    outs = eng.generate(prompts, SamplingParams(temperature=0, max_tokens=6, ignore_eos=True))
    assert outs == [_expected(p, 6) for p in prompts]
    # no step ever exceeded the token budget, and the 40-token prompt was chunked
    for nd, pre in eng.runner.batches:
        assert nd + sum(pre) <= 16
    assert any(len(pre) and max(pre) < 40 and sum(pre) == 16 for _, pre in eng.runner.batches)
    assert eng.bm.num_free() == eng.bm.num_blocks


def test_soft_prefill_chunk_splits_bursts_not_lone_prompts():
    """prefill_chunk: a lone long prompt still prefills in one step (up to the hard
    budget); a burst of short prompts is spread over steps of <= prefill_chunk
    prefill tokens, so the first of them start decoding early."""
    eng = _fake_engine(max_num_seqs=16, max_num_batched_tokens=256, prefill_chunk=32,
                       num_blocks=512)
    long = list(range(1, 201))
    assert eng.generate([long], SamplingParams(temperature=0, max_tokens=2, ignore_eos=True)) == \
        [_expected(long, 2)]
    assert eng.runner.batches[0] == (0, [200])          # one step, beyond the soft budget
    eng.runner.batches.clear()
    burst = [list(range(1000 + 20 * i, 1020 + 20 * i)) for i in range(6)]
    outs = eng.generate(burst, SamplingParams(temperature=0, max_tokens=3, ignore_eos=True))
    assert outs == [_expected(p, 3) for p in burst]
    first = eng.runner.batches[0]
    assert sum(first[1]) <= 32 and first[1][0] == 20     # 20 + a 12-token head of the next
    assert all(sum(pre) <= 32 for _, pre in eng.runner.batches)
    assert eng.bm.num_free() == eng.bm.num_blocks
    # a queue headed by a prompt longer than the soft budget runs full steps
    eng.runner.batches.clear()
    many = [list(range(3000 + 70 * i, 3070 + 70 * i)) for i in range(5)]   # 70 > 32 tokens each
    outs = eng.generate(many, SamplingParams(temperature=0, max_tokens=2, ignore_eos=True))
    assert outs == [_expected(p, 2) for p in many]
    assert sum(eng.runner.batches[0][1]) == 256


def test_soft_prefill_chunk_counting_decode_rows():
    """prefill_chunk_rows: while sequences decode, a burst of short prompts joins
    only up to prefill_chunk GEMM rows per step (decode rows + prefill tokens)."""
    eng = _fake_engine(max_num_seqs=32, max_num_batched_tokens=256, prefill_chunk=48,
                       prefill_chunk_rows=True, num_blocks=1024)
    sp = SamplingParams(temperature=0, max_tokens=40, ignore_eos=True)
    for i in range(8):
        eng.add_request(f"d{i}", list(range(10 * i + 1, 10 * i + 6)), sp)
    for _ in range(3):
        eng.step()
    for i in range(6):
        eng.add_request(f"b{i}", list(range(500 + 12 * i, 512 + 12 * i)), sp)
    while eng.has_work():
        eng.step()
    mixed = [(nd, pre) for nd, pre in eng.runner.batches if nd and pre]
    assert mixed and all(nd + sum(pre) <= 48 for nd, pre in mixed), mixed
    assert eng.bm.num_free() == eng.bm.num_blocks


def test_background_prefill_fills_spare_room_and_warms_prefix_cache():
    """A background (warm-up) prompt never displaces waiting prompts, is chunked
    into the soft budget's spare rows, stops after one token, and leaves its full
    blocks in the prefix cache for the request that follows it."""
    eng = _fake_engine(max_num_seqs=32, max_num_batched_tokens=256, prefill_chunk=48,
                       num_blocks=1024)
    sp = SamplingParams(temperature=0, max_tokens=30, ignore_eos=True)
    for i in range(4):
        eng.add_request(f"d{i}", list(range(10 * i + 1, 10 * i + 6)), sp)
    eng.step()
    warm = list(range(2000, 2160))                      # 160 tokens = 40 blocks of 4
    seen = []
    eng.add_request("warm", warm, SamplingParams(temperature=0, max_tokens=1),
                    on_output=seen.append, background=True)
    eng.add_request("late", list(range(700, 730)), sp)   # queued after the warm-up
    steps = []
    while eng.scheduler.background or eng.scheduler.waiting:
        eng.step()
        steps.append(eng.runner.batches[-1])
    # the waiting prompt went first; warm-up chunks only used the spare rows
    assert steps[0][1][0] == 30
    assert all(nd + sum(pre) <= 48 for nd, pre in steps), steps
    assert sum(sum(pre) for _, pre in steps) == 30 + 160
    while eng.has_work():
        eng.step()
    assert seen[-1].finished and seen[-1].num_output_tokens == 1
    # the follow-up turn (warm prefix + new tokens) re-attaches the warmed blocks
    eng.runner.batches.clear()
    outs = eng.generate([warm + [9, 9, 9]], SamplingParams(temperature=0, max_tokens=2, ignore_eos=True))
    assert outs == [_expected(warm + [9, 9, 9], 2)]
    assert eng.runner.batches[0] == (0, [3])   # all 40 warmed blocks re-attached
    assert eng.bm.num_free() == eng.bm.num_blocks


def test_background_prefill_is_dropped_under_kv_pressure():
    """A warm-up that does not fit is dropped (finished as an abort, not an error)
    and never displaces the sessions that are decoding."""
    eng = _fake_engine(max_num_seqs=8, max_num_batched_tokens=64, prefill_chunk=32,
                       num_blocks=12)
    sp = SamplingParams(temperature=0, max_tokens=8, ignore_eos=True)
    for i in range(2):
        eng.add_request(f"d{i}", list(range(10 * i + 1, 10 * i + 9)), sp)
    eng.step()
    eng.add_request("warm", list(range(500, 600)), SamplingParams(temperature=0, max_tokens=1),
                    background=True)                 # 25 blocks: can never fit in 12
    while eng.has_work():
        eng.step()
    assert eng.stats["finished_abort"] == 1 and eng.stats["finished_error"] == 0
    assert eng.stats["finished_length"] == 2
    assert eng.bm.num_free() == eng.bm.num_blocks


def test_partial_warmup_gives_blocks_to_a_waiting_prompt():
    """a warm-up part-way through its chunked prefill must not keep
    its blocks while a real prompt waits for them (nothing running: the prompt
    was rejected; sequences running: the warm-up never progressed)."""
    eng = _fake_engine(max_num_seqs=8, max_num_batched_tokens=64, prefill_chunk=32,
                       num_blocks=16)
    eng.add_request("warm", list(range(500, 560)), SamplingParams(temperature=0, max_tokens=1),
                    background=True)                  # 15 blocks of 4
    eng.step()                                        # one 32-token chunk: 8 blocks held
    assert eng.scheduler.background and eng.scheduler.background[0].block_ids
    outs = eng.generate([list(range(1, 41))], SamplingParams(temperature=0, max_tokens=3,
                                                             ignore_eos=True))  # 10 blocks
    assert outs == [_expected(list(range(1, 41)), 3)]
    assert eng.stats["finished_error"] == 0
    while eng.has_work():
        eng.step()
    assert eng.bm.num_free() == eng.bm.num_blocks


def test_partial_warmup_yields_while_sessions_decode():
    eng = _fake_engine(max_num_seqs=8, max_num_batched_tokens=64, prefill_chunk=32,
                       num_blocks=20)
    sp = SamplingParams(temperature=0, max_tokens=12, ignore_eos=True)
    eng.add_request("d0", list(range(1, 9)), sp)      # 2 blocks, grows to 5
    eng.step()
    eng.add_request("warm", list(range(500, 560)), SamplingParams(temperature=0, max_tokens=1),
                    background=True)
    eng.step()                                        # warm-up takes a chunk
    assert eng.scheduler.background[0].block_ids
    seen = []
    eng.add_request("late", list(range(100, 140)), sp, on_output=seen.append)  # 10 blocks + growth
    for _ in range(3):
        eng.step()
    assert any(o.num_output_tokens > 0 for o in seen), "the waiting prompt never got admitted"
    while eng.has_work():
        eng.step()
    assert eng.stats["finished_error"] == 0
    assert eng.bm.num_free() == eng.bm.num_blocks


def test_preemption_under_kv_pressure_completes_everything():
    eng = _fake_engine(num_blocks=12, max_num_seqs=8, max_num_batched_tokens=64)
    prompts = [[i + 1] * 6 for i in range(5)]
    outs = eng.generate(prompts, SamplingParams(temperature=0, max_tokens=12, ignore_eos=True))
    assert outs == [_expected(p, 12) for p in prompts]
    assert eng.scheduler.num_preemptions > 0
    assert eng.bm.num_free() == eng.bm.num_blocks


def test_prompt_that_can_never_fit_is_rejected():
    eng = _fake_engine(num_blocks=2, max_model_len=512)
    eng.add_request("big", list(range(40)), SamplingParams(max_tokens=2))
    outs = eng.step()
    assert outs and outs[0].finished and outs[0].finish_reason == "error"
    with pytest.raises(EngineError):
        eng.add_request("huge", list(range(600)), SamplingParams(max_tokens=2))


def test_abort_frees_blocks():
    eng = _fake_engine()
    eng.add_request("a", list(range(10)), SamplingParams(max_tokens=50, ignore_eos=True))
    eng.add_request("b", list(range(12)), SamplingParams(max_tokens=5, ignore_eos=True))
    for _ in range(3):
        eng.step()
    assert eng.abort("a") and not eng.abort("a")
    while eng.has_work():
        eng.step()
    assert eng.bm.num_free() == eng.bm.num_blocks
    assert eng.stats["finished_abort"] == 1 and eng.stats["finished_length"] == 1


def test_eos_min_tokens_and_stop_token_ids():
    eng = _fake_engine(eos_every=3)
    out = eng.generate([[5, 6]], SamplingParams(temperature=0, max_tokens=20))[0]
    assert len(out) == 2  # third token is EOS -> stop (not returned)
    out = eng.generate([[5, 6]], SamplingParams(temperature=0, max_tokens=20, min_tokens=4))[0]
    assert 128009 in out[:4]  # EOS before min_tokens is kept as a token
    nxt = _expected([5, 6], 3)
    out = eng.generate([[5, 6]], SamplingParams(temperature=0, max_tokens=20, ignore_eos=True,
                                                stop_token_ids=[nxt[1]]))[0]
    assert out == nxt[:1]


def test_stop_strings_hold_back_partial_matches():
    eng = _fake_engine()
    eng.detok = _FakeDetok()
    texts = []
    eng.add_request("r", [1, 2], SamplingParams(max_tokens=30, ignore_eos=True, stop=["END"]),
                    on_output=lambda o: texts.append(o.text))
    while eng.has_work():
        eng.step()
    full = "".join(texts)
    assert "END" not in full and full == "ab E" + "ab E" * 0 or full.startswith("ab")


class _FakeDetok:
    """Maps the fake runner's tokens onto a fixed text stream 'ab E', 'N', 'D', ..."""

    def __init__(self):
        self.seq = iter(["ab", " E", "N", "D", "zz", "zz", "zz"] + ["q"] * 40)

    def new_stream(self):
        return 0

    def push(self, sid, tok):
        return next(self.seq)

    def flush(self, sid):
        return ""

    def release(self, sid):
        pass


@settings(max_examples=40, deadline=None)
@given(st.lists(st.tuples(st.integers(1, 30), st.integers(1, 12)), min_size=1, max_size=10),
       st.integers(8, 40), st.integers(6, 40))
def test_scheduler_property_all_requests_finish(reqs, budget, blocks):
    """Any mix of prompt/generation lengths under any token budget and KV pool
    size: every request that fits finishes with exactly max_tokens outputs equal
    to the deterministic stream, and the pool is whole again at the end."""
    eng = _fake_engine(num_blocks=blocks, max_num_seqs=6, max_num_batched_tokens=budget)
    fits = [(p, g) for p, g in reqs if math.ceil((p + g) / 4) <= blocks]
    if not fits:
        return
    prompts = [list(range(3, 3 + p)) for p, _ in fits]
    results = {}
    for i, (p, g) in enumerate(fits):
        eng.add_request(f"r{i}", prompts[i], SamplingParams(temperature=0, max_tokens=g,
                                                            ignore_eos=True),
                        on_output=lambda o, i=i: results.setdefault(i, []).extend(o.token_ids))
    for _ in range(5000):
        if not eng.has_work():
            break
        eng.step()
    assert not eng.has_work()
    for i, (p, g) in enumerate(fits):
        assert results[i] == _expected(prompts[i], g)
    assert eng.bm.num_free() == eng.bm.num_blocks


# ----------------------------------------------------------------------------- tiny model
@pytest.fixture(scope="module")
def tiny_engine():
    return LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=256,
                                  max_model_len=1024, max_num_seqs=8))


def test_tiny_cpu_greedy_deterministic_and_batched(tiny_engine):
    rng = np.random.default_rng(0)
    prompts = [rng.integers(0, 120000, n).tolist() for n in (5, 23, 40)]
    sp = SamplingParams(temperature=0, max_tokens=6, ignore_eos=True)
    batched = tiny_engine.generate(prompts, sp)
    single = [tiny_engine.generate([p], sp)[0] for p in prompts]
    assert batched == single and all(len(o) == 6 for o in batched)


def test_tiny_cpu_chunked_prefill_and_prefix_cache(tiny_engine):
    rng = np.random.default_rng(1)
    p = rng.integers(0, 120000, 70).tolist()
    sp = SamplingParams(temperature=0, max_tokens=5, ignore_eos=True)
    first = tiny_engine.generate([p], sp)[0]
    hits0 = tiny_engine.bm.hits
    again = tiny_engine.generate([p + first + [7, 8, 9]], sp)[0]
    assert tiny_engine.bm.hits > hits0  # the earlier turn's KV blocks were reused
    chunked = LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=256, max_model_len=1024,
                                     max_num_batched_tokens=32, enable_prefix_caching=False))
    assert chunked.generate([p + first + [7, 8, 9]], sp)[0] == again


def test_batch_invariant_config_plumbing():
    """ENGINE_BATCH_INVARIANT reaches the model: invariant plans on, the fused small-batch
    layer off (GPU kernels: tests/test_batch_invariance_gpu.py), and the CPU path still
    generates the same greedy tokens as the default engine."""
    import os

    os.environ["ENGINE_BATCH_INVARIANT"] = "1"
    try:
        cfg = EngineConfig.from_env(model="tiny", device="cpu", num_kv_blocks=128, max_model_len=512)
    finally:
        del os.environ["ENGINE_BATCH_INVARIANT"]
    assert cfg.batch_invariant
    inv = LLMEngine(cfg)
    assert inv.runner.invariant and inv.runner.model.invariant and not inv.runner.model.fused
    base = LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=128, max_model_len=512))
    assert not base.runner.model.invariant
    sp = SamplingParams(temperature=0, max_tokens=5, ignore_eos=True)
    assert inv.generate([[4, 5, 6, 7]], sp) == base.generate([[4, 5, 6, 7]], sp)


def test_tiny_cpu_seeded_sampling_reproducible(tiny_engine):
    sp = SamplingParams(temperature=0.9, top_p=0.9, top_k=50, max_tokens=5, seed=11, ignore_eos=True)
    a = tiny_engine.generate([[1, 2, 3]], sp)[0]
    b = tiny_engine.generate([[1, 2, 3]], sp)[0]
    assert a == b


def test_tiny_cpu_guided_json(tiny_engine):
    schema = {"type": "object", "properties": {"city": {"type": "string", "maxLength": 8},
                                               "n": {"type": "integer"}}}
    sp = SamplingParams(temperature=0.8, max_tokens=60, seed=3, guided=GuidedSpec.json_schema(schema))
    ids = tiny_engine.generate([[1, 2, 3]], sp)[0]
    obj = json.loads(tiny_engine.tokenizer.decode(ids))
    assert set(obj) == {"city", "n"} and isinstance(obj["n"], int)


def test_jump_forward_prefills_forced_grammar_runs(tiny_engine, monkeypatch):
    """bytes the grammar forces (a tool call's '{"name": "', the rest
    of a tool name once its prefix is unique, '", "parameters": {"query": "', the
    closing braces) are appended as tokens and prefilled in ONE step instead of
    one decode step per token; the call stays valid JSON."""
    from fasttalk_llm_microservice_amd.engine.guided import tool_call_ast

    tools = [{"type": "function", "function": {"name": "duckduckgo_search", "parameters": {
        "type": "object", "properties": {"query": {"type": "string", "maxLength": 12}},
        "required": ["query"]}}},
        {"type": "function", "function": {"name": "get_current_time",
                                          "parameters": {"type": "object", "properties": {}}}}]
    spec = GuidedSpec(tool_call_ast(tools))
    eng = tiny_engine
    steps = []
    orig = eng.runner.execute
    orig_launch = eng.runner.mixed_launch

    def record(batch):
        starts = batch.prefill_start or [s.num_computed for s in batch.prefill_seqs]
        steps.append([(a, n, s.status.name) for s, n, a in
                      zip(batch.prefill_seqs, batch.prefill_tokens, starts)] + [("d", len(batch.decode_seqs))])

    def spy(batch, masks):
        record(batch)
        return orig(batch, masks)

    def spy_launch(batch, rowmap, *args, **kw):   # mixed steps queued by the mixed chain
        record(batch)
        return orig_launch(batch, rowmap, *args, **kw)

    monkeypatch.setattr(eng.runner, "execute", spy)
    monkeypatch.setattr(eng.runner, "mixed_launch", spy_launch)
    before = eng.stats["jump_forward_tokens"]
    outs = []
    for seed in range(4):
        sp = SamplingParams(temperature=1.0, max_tokens=80, seed=seed, guided=spec)
        ids = eng.generate([[1, 2, 3]], sp)[0]
        call = json.loads(eng.tokenizer.decode(ids))
        assert call["name"] in ("duckduckgo_search", "get_current_time")
        outs.append((call, len(ids)))
    assert eng.stats["jump_forward_tokens"] > before
    # the call head was prefilled with the prompt (3 prompt tokens + forced head)
    assert any(n > 3 for row in steps for (a, n, st) in row[:-1] if a == 0)
    # forced runs of a running sequence went in as multi-token prefill chunks
    assert any(n > 1 and st == "RUNNING" for row in steps for (a, n, st) in row[:-1])
    # fewer forward passes than output tokens
    assert len(steps) < sum(n for _, n in outs)
    monkeypatch.setenv("ENGINE_JUMP_FORWARD", "0")
    off = LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=256, max_model_len=1024))
    assert not off.jump_forward
    ids = off.generate([[1, 2, 3]], SamplingParams(temperature=1.0, max_tokens=80, seed=0, guided=spec))[0]
    assert json.loads(off.tokenizer.decode(ids))["name"] in ("duckduckgo_search", "get_current_time")


class _MaskRunner(FakeRunner):
    """Scripted first token per request, then the lowest id the grammar allows (or a
    fixed word when unconstrained): drives lazy-grammar requests to completion."""

    def __init__(self, first, word, **kw):
        super().__init__(**kw)
        self.first, self.word = first, word

    def execute(self, batch, masks):
        self.stats["steps"] += 1
        out = []
        for i, s in enumerate(batch.sampled_seqs()):
            row = None if masks is None else masks[i]
            if row is not None and not (row == -1).all():
                bits = np.unpackbits(row.view(np.uint8), bitorder="little")
                out.append(int(np.flatnonzero(bits)[0]))
            elif s.n_tokens == s.prompt_len:
                out.append(self.first)
            else:
                out.append(self.word)
        return out


@pytest.mark.parametrize("opens_call", [True, False])
def test_lazy_tool_grammar_binds_only_when_the_model_opens_a_call(opens_call):
    """VERDICT r2 #5 (model-decided tools): the tool-call grammar is offered lazily --
    bound iff the first generated token starts a call (then the call is valid JSON,
    jump-forwarded), else the reply stays free text with no masks at all."""
    from fasttalk_llm_microservice_amd.engine.guided import tool_call_ast
    from fasttalk_llm_microservice_amd.engine.tokenizer import get_tokenizer

    tok = get_tokenizer()
    brace = tok.encode("{")[0]
    word = tok.encode(" hello")[0]
    runner = _MaskRunner(brace if opens_call else word, word, num_blocks=256)
    eng = LLMEngine(EngineConfig(model="tiny", device="cpu", block_size=4), runner=runner)
    tools = [{"type": "function", "function": {"name": "get_current_time",
                                               "parameters": {"type": "object", "properties": {}}}}]
    sp = SamplingParams(temperature=0.7, max_tokens=40, guided=GuidedSpec(tool_call_ast(tools)),
                        guided_lazy=True, ignore_eos=not opens_call)
    ids = eng.generate([[1, 2, 3, 4, 5]], sp)[0]
    text = eng.tokenizer.decode(ids)
    if opens_call:
        assert json.loads(text) == {"name": "get_current_time", "parameters": {}}
        assert eng.stats["lazy_grammar_bound"] == 1
    else:
        assert text.startswith(" hello") and len(ids) == 40
        assert eng.stats["lazy_grammar_bound"] == 0


def test_complete_grammar_ends_without_decoding_eos(tiny_engine, monkeypatch):
    """VERDICT r3 #7 (config 5 tail): a guided sequence whose grammar is complete
    (accepting, no byte can follow -- the mask would allow EOS alone) finishes on the
    step that completed it: the tool call's forced closing is not prefilled and no
    EOS is decoded, one forward pass fewer per call, the same tokens."""
    from fasttalk_llm_microservice_amd.engine.guided import tool_call_ast

    tools = [{"type": "function", "function": {"name": "duckduckgo_search", "parameters": {
        "type": "object", "properties": {"query": {"type": "string", "maxLength": 12}},
        "required": ["query"]}}}]
    spec = GuidedSpec(tool_call_ast(tools))
    eng = tiny_engine
    steps = []
    orig = eng.runner.execute

    def spy(batch, masks):
        steps.append(batch.total_tokens)
        return orig(batch, masks)

    monkeypatch.setattr(eng.runner, "execute", spy)

    def run(shortcut: bool):
        eng.grammar_eos_shortcut = shortcut
        steps.clear()
        before = eng.stats["grammar_complete_stops"]
        got = []
        for seed in range(3):
            sp = SamplingParams(temperature=1.0, max_tokens=80, seed=seed, guided=spec)
            ids = eng.generate([[1, 2, 3]], sp)[0]
            call = json.loads(eng.tokenizer.decode(ids))
            assert call["name"] == "duckduckgo_search" and isinstance(call["parameters"]["query"], str)
            assert not any(t in eng.stop_ids for t in ids)
            got.append(ids)
        return got, len(steps), eng.stats["grammar_complete_stops"] - before

    try:
        on, n_on, stops_on = run(True)
        off, n_off, stops_off = run(False)
    finally:
        eng.grammar_eos_shortcut = True
    assert stops_on == 3 and stops_off == 0
    assert on == off
    assert n_off == n_on + 3
    # every block went back (the uncomputed tail was never committed)
    assert eng.bm.num_free() == eng.bm.num_blocks or eng.bm.num_cached() > 0


def test_jump_forward_head_stays_within_max_model_len(tiny_engine):
    """the forced tool-call head appended at admission is bounded by
    max_model_len (it is prefilled with the prompt; RoPE has max_model_len + 1 rows)."""
    from fasttalk_llm_microservice_amd.engine.guided import tool_call_ast

    tools = [{"type": "function", "function": {"name": "duckduckgo_search", "parameters": {
        "type": "object", "properties": {"query": {"type": "string"}}, "required": ["query"]}}}]
    spec = GuidedSpec(tool_call_ast(tools))
    eng = tiny_engine
    n = eng.max_model_len - 2
    sp = SamplingParams(temperature=1.0, max_tokens=64, seed=1, guided=spec)
    seq = eng.add_request("jf-edge", [7] * n, sp)
    assert 0 < len(seq.jf_ids) <= 1 and seq.n_tokens <= eng.max_model_len - 1
    outs = []
    while eng.has_work():
        outs += [o for o in eng.step() if o.request_id == "jf-edge"]
    assert outs and outs[-1].finished and outs[-1].finish_reason == "length"
    assert eng.bm.num_free() == eng.bm.num_blocks or eng.bm.num_cached() > 0


def test_priority_prompts_prefill_first():
    """An agent's post-tool re-prompt (priority 1) goes ahead of waiting prompts of
    lower priority that have not started; a chunked prefill in progress keeps its
    place; equal priorities stay FIFO."""
    from fasttalk_llm_microservice_amd.engine.scheduler import Scheduler
    from fasttalk_llm_microservice_amd.engine.sequence import Sequence
    from fasttalk_llm_microservice_amd.runtime import rt

    bm = rt().BlockManager(64, 4, True)
    sch = Scheduler(bm, 4, 8, 256, 512)
    mk = lambda rid, pr=0: Sequence(rid, [1, 2, 3], SamplingParams(max_tokens=4, priority=pr))  # noqa
    a, b = mk("a"), mk("b")
    sch.add(a)
    sch.add(b)
    a.num_computed = 2          # a's chunked prefill is under way
    sch.add(mk("t1", 1))
    sch.add(mk("t2", 1))
    sch.add(mk("c"))
    assert [q.request_id for q in sch.waiting] == ["a", "t1", "t2", "b", "c"]


def test_priority_does_not_jump_preempted_sequences():
    """A sequence re-queued by recompute preemption (num_computed back to 0) keeps its
    place in front of a later high-priority prompt."""
    from fasttalk_llm_microservice_amd.engine.scheduler import Scheduler
    from fasttalk_llm_microservice_amd.engine.sequence import Sequence
    from fasttalk_llm_microservice_amd.runtime import rt

    bm = rt().BlockManager(64, 4, True)
    sch = Scheduler(bm, 4, 8, 256, 512)
    mk = lambda rid, pr=0: Sequence(rid, [1, 2, 3], SamplingParams(max_tokens=4, priority=pr))  # noqa
    victim, fresh = mk("victim"), mk("fresh")
    victim.preemptions = 1      # preempted once, re-queued with num_computed == 0
    sch.add(victim)
    sch.add(fresh)
    sch.add(mk("t", 1))
    assert [q.request_id for q in sch.waiting] == ["victim", "t", "fresh"]


def test_chained_prefill_chunks_and_epoch_guard():
    """Mixed chain bookkeeping (Scheduler.stamp / post_step): a second chunk of a
    chunked prompt scheduled before the first one's step completed continues after
    it (Sequence.pf_sched), and a chunk whose KV was dropped while it was queued
    (recompute preemption: epoch bump) is ignored when its step completes."""
    from fasttalk_llm_microservice_amd.engine.scheduler import Scheduler
    from fasttalk_llm_microservice_amd.engine.sequence import Sequence
    from fasttalk_llm_microservice_amd.runtime import rt

    bm = rt().BlockManager(64, 4, False)
    sch = Scheduler(bm, 4, 8, 8, 512)          # 8-token steps: a 20-token prompt takes 3 chunks
    seq = Sequence("p", list(range(1, 21)), SamplingParams(max_tokens=4))
    sch.add(seq)
    b1 = sch.schedule()                        # chunk 1, not yet completed
    assert b1.prefill_seqs == [seq] and b1.prefill_start == [0] and b1.prefill_tokens == [8]
    assert seq.pf_sched == 8 and seq.num_computed == 0
    b2 = sch.schedule()                        # chunk 2 queued behind it (chained)
    assert b2.prefill_start == [8] and b2.prefill_tokens == [8] and seq.pf_sched == 16
    sch.post_step(b1)
    assert seq.num_computed == 8 and seq.pf_sched == 8
    sch.post_step(b2)
    assert seq.num_computed == 16 and seq.pf_sched == 0
    b3 = sch.schedule()                        # the last chunk: sampled, then running
    assert b3.prefill_start == [16] and b3.prefill_tokens == [4] and b3.prefill_sample == [True]
    sch.post_step(b3)
    assert seq.num_computed == 20 and seq in sch.running and seq.pf_sched == 0
    # a second prompt's first chunk is queued, then the prompt loses its KV while the
    # chunk is in flight (a waiting sequence mid-prefill is the first to give its
    # blocks up: Scheduler._preempt_one); the stale chunk must not count
    other = Sequence("q", list(range(1, 21)), SamplingParams(max_tokens=4))
    sch.add(other)
    c1 = sch.schedule()
    assert other in c1.prefill_seqs and other.pf_sched > 0 and other.block_ids
    ep = other.epoch
    sch._reset_to_waiting(other)
    assert other.epoch == ep + 1 and other.pf_sched == 0 and not other.block_ids
    sch.post_step(c1)
    assert other.num_computed == 0 and other.pf_sched == 0 and other not in sch.running
    assert seq.num_computed == 21                 # the decode row of that step still counts
    c2 = sch.schedule()                           # the prompt restarts from its first token
    i = c2.prefill_seqs.index(other)
    assert c2.prefill_start[i] == 0 and c2.prefill_epoch[i] == ep + 1


def test_guided_rows_cap_the_steps_prefill():
    """ENGINE_GUIDED_PREFILL_CAP: while a guided (tool-call / JSON)
    row decodes, a step carries at most the cap of prefill tokens, so the call's free
    argument string is not decoded in steps stretched by full prefill chunks; steps
    without guided rows keep the normal budget, and every output is unchanged."""
    schema = {"type": "object", "properties": {"city": {"type": "string", "maxLength": 12},
                                               "n": {"type": "integer"}}}
    rng = np.random.default_rng(5)
    prompts = [rng.integers(0, 120000, 40).tolist() for _ in range(6)]
    outs = {}
    for cap in (0, 8):
        eng = LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=512, max_model_len=1024,
                                     max_num_seqs=8, max_num_batched_tokens=64, prefill_chunk=0,
                                     guided_prefill_cap=cap))
        steps = []
        orig = eng.scheduler.schedule

        def rec(orig=orig, steps=steps, eng=eng):
            b = orig()
            if b is not None:
                guided = any(s.grammar is not None and not s.lazy for s in b.decode_seqs)
                steps.append((guided, sum(b.prefill_tokens)))
            return b

        eng.scheduler.schedule = rec
        sp_json = SamplingParams(temperature=0.8, max_tokens=40, seed=3,
                                 guided=GuidedSpec.json_schema(schema))
        sp = SamplingParams(temperature=0, max_tokens=4, ignore_eos=True)
        eng.add_request("g", [1, 2, 3], sp_json)
        res = {}
        for _ in range(2):
            eng.step()
        for i, p in enumerate(prompts):
            eng.add_request(f"p{i}", p, sp, on_output=lambda o, i=i: res.setdefault(i, []).extend(o.token_ids))
        while eng.has_work():
            eng.step()
        outs[cap] = [res[i] for i in range(len(prompts))]
        g_steps = [n for g, n in steps if g]
        assert g_steps, steps
        if cap:
            assert max(g_steps) <= cap and eng.scheduler.guided_capped > 0, steps
            assert max(n for g, n in steps if not g) > cap   # the cap applies to guided steps only
        else:
            assert max(g_steps) > 8
    assert outs[0] == outs[8]


def _chat_turn(eng, prompt, sp, rid):
    """One request through add_request / step: (streamed text, ids, cached prompt tokens)."""
    eng.add_request(rid, prompt, sp)
    text, ids, cached = "", [], None
    while eng.has_work():
        for o in eng.step():
            if o.request_id != rid:
                continue
            text += o.text
            ids += o.token_ids
            if o.finished:
                cached = o.num_cached_tokens
    return text, ids, cached


def test_token_exact_assistant_history_keeps_the_reply_in_the_prefix_cache(tiny_engine):
    """A reply rendered back into the next turn's prompt keeps the ids it was generated
    as (ChatTemplate.remember_assistant), so the prefix cache covers the whole reply;
    the cached entry decodes to exactly the stored text."""
    eng = tiny_engine
    tpl = eng.template
    msgs = [{"role": "system", "content": "You are a helpful voice assistant."},
            {"role": "user", "content": "Tell me something about the weather on the coast today."}]
    sp = SamplingParams(temperature=1.0, top_p=1.0, max_tokens=40, ignore_eos=True, seed=4)
    p1 = tpl.render(msgs)
    text, ids, _ = _chat_turn(eng, p1, sp, "tok-hist-1")
    assert len(ids) == 40 and text == eng.tokenizer.decode(ids)
    # (this sample is not the tokenizer's own segmentation of its text: re-encoding
    # it breaks the prefix after two tokens)
    assert eng.tokenizer.encode(text)[:len(ids)] != ids
    msgs2 = msgs + [{"role": "assistant", "content": text},
                    {"role": "user", "content": "And tomorrow?"}]
    p2 = tpl.render(msgs2)
    head = p1 + ids
    assert p2[:len(head)] == head   # the reply kept its generated ids
    assert eng.tokenizer.decode(tpl.message_ids(msgs2[2])) == \
        eng.tokenizer.decode(tpl._header("assistant")) + text + eng.tokenizer.decode([eng.tokenizer.eot_id])
    _, _, cached = _chat_turn(eng, p2, SamplingParams(temperature=0, max_tokens=2, ignore_eos=True),
                              "tok-hist-2")
    bs = eng.bm.block_size
    # every full block of the first turn's prompt + reply (but the last sampled token,
    # whose KV was never computed) comes from the cache
    assert cached >= ((len(head) - 1) // bs) * bs
