"""Host KV swap (E6 / K13, vLLM ``--swap-space``, ``docker-compose.vllm.yml:49``).

A fake runner keeps a token-id "KV cache" per block and checks, on every step,
that each scheduled sequence's blocks hold exactly the tokens it attends over:
that is the invariant swap-out / swap-in, prefix re-attachment on swap-in and
block reuse inside a swapping step must preserve.  The tiny CPU model then
checks that a generation that was swapped out and back produces the same tokens
(greedy and seeded sampling) as one that never was."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams

from test_engine_cpu import FakeRunner, _expected

BS = 4


class KVFakeRunner(FakeRunner):
    def __init__(self, num_blocks=16, num_host_blocks=32, **kw):
        super().__init__(num_blocks=num_blocks, **kw)
        self.num_host_blocks = num_host_blocks
        self.kv = np.full((num_blocks, BS), -1, np.int64)
        self.host = np.full((max(num_host_blocks, 1), BS), -1, np.int64)
        self.swaps = 0

    def swap(self, swap_out, swap_in):
        self.swaps += 1
        for d, h in swap_out:
            self.host[h] = self.kv[d]
        for h, d in swap_in:
            self.kv[d] = self.host[h]

    def _check_and_write(self, seq, n_new):
        toks = seq.tokens
        for pos in range(seq.num_computed):
            b = seq.block_ids[pos // BS]
            assert self.kv[b, pos % BS] == toks[pos], \
                f"{seq.request_id}: KV of position {pos} is stale"
        for pos in range(seq.num_computed, seq.num_computed + n_new):
            self.kv[seq.block_ids[pos // BS], pos % BS] = toks[pos]

    def execute(self, batch, masks):
        for s in batch.decode_seqs:
            self._check_and_write(s, 1)
        for s, n in zip(batch.prefill_seqs, batch.prefill_tokens):
            self._check_and_write(s, n)
        return super().execute(batch, masks)


def _engine(num_blocks, host_blocks, **kw):
    cfg = EngineConfig(model="tiny", device="cpu", block_size=BS, **kw)
    return LLMEngine(cfg, runner=KVFakeRunner(num_blocks=num_blocks, num_host_blocks=host_blocks))


def test_swap_preemption_keeps_kv_and_outputs():
    eng = _engine(12, 32, max_num_seqs=8, max_num_batched_tokens=64)
    prompts = [[i + 1] * 6 for i in range(5)]
    outs = eng.generate(prompts, SamplingParams(temperature=0, max_tokens=12, ignore_eos=True))
    assert outs == [_expected(p, 12) for p in prompts]
    s = eng.scheduler
    assert s.num_swap_out > 0 and s.num_swap_in == s.num_swap_out
    assert eng.runner.swaps > 0 and eng.stats["swapped_in_blocks"] > 0
    assert eng.bm.num_free() == eng.bm.num_blocks and s.host.num_free() == s.host.num_blocks


def test_swap_falls_back_to_recompute_when_host_pool_is_full():
    eng = _engine(12, 2, max_num_seqs=8, max_num_batched_tokens=64)
    prompts = [[i + 1] * 6 for i in range(5)]
    outs = eng.generate(prompts, SamplingParams(temperature=0, max_tokens=12, ignore_eos=True))
    assert outs == [_expected(p, 12) for p in prompts]
    assert eng.scheduler.host.num_free() == 2


def test_abort_of_swapped_sequence_frees_host_slots():
    eng = _engine(8, 32, max_num_seqs=8, max_num_batched_tokens=64)
    for i in range(4):
        eng.add_request(f"r{i}", [i + 1] * 6, SamplingParams(max_tokens=40, ignore_eos=True))
    s = eng.scheduler
    for _ in range(60):
        eng.step()
        if s.swapped:
            break
    assert s.swapped, "the pool is too small for 4 sequences: one must be swapped out"
    victim = s.swapped[0]
    assert victim.host_slots and eng.abort(victim.request_id)
    assert not victim.host_slots and victim not in s.swapped
    while eng.has_work():
        eng.step()
    assert eng.bm.num_free() == eng.bm.num_blocks and s.host.num_free() == s.host.num_blocks


@settings(max_examples=60, deadline=None)
@given(st.lists(st.tuples(st.integers(1, 30), st.integers(1, 14)), min_size=1, max_size=10),
       st.integers(8, 48), st.integers(6, 24), st.sampled_from([0, 3, 8, 64]))
def test_swap_property_kv_always_consistent(reqs, budget, blocks, host_blocks):
    eng = _engine(blocks, host_blocks, max_num_seqs=6, max_num_batched_tokens=budget)
    prompts = [[(7 * i + j) % 50 + 1 for j in range(n)] for i, (n, _) in enumerate(reqs)]
    ok = []
    for i, (p, (_, m)) in enumerate(zip(prompts, reqs)):
        eng.add_request(f"q{i}", p, SamplingParams(temperature=0, max_tokens=m, ignore_eos=True),
                        on_output=lambda o, i=i: ok.append(i) if o.finished else None)
    for _ in range(5000):
        if not eng.has_work():
            break
        eng.step()
    assert not eng.has_work()
    assert sorted(ok) == list(range(len(reqs)))
    assert eng.bm.num_free() == eng.bm.num_blocks
    if eng.scheduler.host is not None:
        assert eng.scheduler.host.num_free() == eng.scheduler.host.num_blocks


@pytest.mark.parametrize("temperature", [0.0, 0.8])
def test_tiny_cpu_swap_matches_unconstrained(temperature):
    """Real KV tensors: generation across a swap-out/in reproduces the tokens of a
    run with memory to spare (the sampling stream continues: a swap is not a
    recompute preemption)."""
    prompts = [[(5 * i + j) % 300 + 1 for j in range(20)] for i in range(4)]
    sp = SamplingParams(temperature=temperature, top_p=0.9, max_tokens=24, ignore_eos=True,
                        seed=11)
    big = LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=256,
                                 max_model_len=512, block_size=16))
    ref = big.generate(prompts, sp)
    small = LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=7, max_model_len=512,
                                   block_size=16, swap_space_gb=1.0,
                                   enable_prefix_caching=False))
    got = small.generate(prompts, sp)
    assert small.scheduler.num_swap_out > 0
    assert small.scheduler.num_preemptions == small.scheduler.num_swap_out
    assert got == ref


def test_failed_step_finishes_swapped_sequences():
    """a step failure (e.g. in the swap copy) must also end the swapped
    sequences with an error and give their host slots back -- they must never
    resume on KV that was not copied."""
    eng = _engine(8, 32, max_num_seqs=8, max_num_batched_tokens=64)
    done = {}
    for i in range(4):
        eng.add_request(f"r{i}", [i + 1] * 6, SamplingParams(max_tokens=40, ignore_eos=True),
                        on_output=lambda o: done.__setitem__(o.request_id, o) if o.finished else None)
    s = eng.scheduler
    for _ in range(60):
        eng.step()
        if s.swapped:
            break
    assert s.swapped
    victims = [q.request_id for q in s.swapped]
    eng.fail_unfinished("FT_FAULT: swap copy failed")
    assert not eng.has_work()
    assert all(done[v].finish_reason == "error" for v in victims)
    assert eng.bm.num_free() == eng.bm.num_blocks and s.host.num_free() == s.host.num_blocks


def test_swapped_in_blocks_return_to_the_prefix_cache():
    """blocks restored by a swap-in are committed again, so a follow-up
    turn that shares the prefix hits the cache."""
    eng = _engine(12, 32, max_num_seqs=8, max_num_batched_tokens=64)
    for i in range(5):
        eng.add_request(f"r{i}", [i + 1] * 6, SamplingParams(max_tokens=12, ignore_eos=True))
    s = eng.scheduler
    resumed = None
    for _ in range(200):
        n_in = s.num_swap_in
        before = {q.request_id for q in s.swapped}
        eng.step()
        if s.num_swap_in > n_in:
            resumed = [q for q in s.running if q.request_id in before]
            break
    assert resumed, "no swap-in happened"
    eng.step()  # post_step of the next step commits what the resumed blocks hold
    for seq in resumed:
        nfull = seq.num_computed // BS
        hit = eng.bm.match_prefix(seq.tokens, nfull)
        try:
            assert list(hit) == list(seq.block_ids[:nfull])
        finally:
            eng.bm.free(list(hit))
