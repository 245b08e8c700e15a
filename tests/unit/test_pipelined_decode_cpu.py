"""Pipelined decode (engine.py ``_speculate``) on the CPU with a device-emulating
runner: queued steps take their input ids from the previous queued step's
sampled rows, and a step queued after a sequence is known to have finished
drops that row and gathers the survivors' ids by ``rowmap``.  Tokens must equal
the synchronous engine's exactly (the fake model is deterministic in (input
token, position)), whatever the pipeline depth and however sequences stop."""
import pytest
import torch

from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
from fasttalk_llm_microservice_amd.models.config import MODELS

EOS = 128009


def _next(tok: int, pos: int) -> int:
    if (tok * 31 + pos) % 23 == 0:
        return EOS
    return (tok * 7 + pos * 13 + 3) % 1000 + 1


class _Handle:
    def __init__(self, out):
        self.out = out
        self.event = None


class ModelRunner:
    """Named like the real runner: the engine pipelines only ``ModelRunner``s.
    ``d_out`` plays the device buffer of the last queued step's sampled ids;
    positions come from each sequence's ``inflight`` count, and a queued step
    checks that the KV slot it would write has a block."""

    def __init__(self, num_blocks=256, max_model_len=512, block_size=4):
        self.num_blocks = num_blocks
        self.max_model_len = max_model_len
        self.bs = block_size
        self.mcfg = MODELS["tiny"]
        self.dtype = torch.float32
        self.device = torch.device("cpu")
        self.stats = {"steps": 0}
        self.d_out = []
        self.launches = []   # (rows, ahead, rowmap)
        self.mixed = []      # (decode rows, prefill tokens, rowmap) of queued mixed steps

    def execute(self, batch, masks):
        self.stats["steps"] += 1
        return [_next(int(s.tokens[-1]), s.n_tokens - 1) for s in batch.sampled_seqs()]

    def can_pipeline(self, n: int) -> bool:
        return n > 0

    def step_done(self, h) -> bool:
        return True

    def decode_launch(self, seqs, ahead=0, masks=None, rowmap=None):
        self.launches.append((len(seqs), ahead, None if rowmap is None else list(rowmap)))
        if ahead:
            rows = rowmap if rowmap is not None else range(len(seqs))
            ids = [self.d_out[r] if r >= 0 else int(s.tokens[-1]) for r, s in zip(rows, seqs)]
        else:
            ids = [int(s.tokens[-1]) for s in seqs]
        out = []
        for i, (s, tok) in enumerate(zip(seqs, ids)):
            pos = s.n_tokens - 1 + s.inflight
            assert ahead or s.inflight == 0
            assert not ahead or rowmap is None or rowmap[i] >= 0 or s.inflight == 0
            assert pos // self.bs < len(s.block_ids), "KV slot of a queued step has no block"
            out.append(_next(tok, pos))
        self.d_out = out
        return _Handle(out)

    def decode_collect(self, h):
        return list(h.out)

    def mixed_launch(self, batch, rowmap):
        """``rowmap`` None: launched from a drained queue, ids from the host."""
        self.mixed.append((len(batch.decode_seqs), list(batch.prefill_tokens),
                           None if rowmap is None else list(rowmap)))
        out = []
        for i, s in enumerate(batch.decode_seqs):
            pos = s.n_tokens - 1 + s.inflight
            if rowmap is None or rowmap[i] < 0:
                assert s.inflight == 0
                tok = int(s.tokens[-1])
            else:
                assert s.inflight >= 1
                tok = self.d_out[rowmap[i]]
            assert pos // self.bs < len(s.block_ids)
            out.append(_next(tok, pos))
        starts = batch.prefill_start or [s.num_computed for s in batch.prefill_seqs]
        chunks = self.__dict__.setdefault("chunks", {})
        for s, n, smp, a in zip(batch.prefill_seqs, batch.prefill_tokens, batch.prefill_sample, starts):
            assert s.inflight == 0
            assert (a + n + self.bs - 1) // self.bs <= len(s.block_ids)
            # a prompt's chunks are contiguous, also when queued behind each other
            prev = chunks.get(id(s))
            assert prev is None or prev == a or a == s.num_computed, (prev, a, s.num_computed)
            chunks[id(s)] = a + n
            if smp:
                assert a + n == s.n_tokens
                out.append(_next(int(s.tokens[-1]), s.n_tokens - 1))
        self.d_out = out
        return _Handle(out)

    def mixed_collect(self, h):
        return list(h.out)


def _run(async_output: bool, depth: int, n_req: int = 9, shrink: bool = True, late: int = 0,
         mixed_ahead: bool = False, chain: bool = False, prefill_chunk: int = 512,
         max_batched: int = 8192, num_blocks: int = 256):
    """``late`` requests arrive one every third engine step after the first ``n_req``."""
    import os

    os.environ["ENGINE_PIPELINE_SHRINK"] = "1" if shrink else "0"
    os.environ["ENGINE_MIXED_AHEAD"] = "1" if mixed_ahead else "0"
    os.environ["ENGINE_MIXED_CHAIN"] = "1" if chain else "0"
    cfg = EngineConfig(model="tiny", device="cpu", block_size=4, async_output=async_output,
                       pipeline_depth=depth, max_num_seqs=32, prefill_chunk=prefill_chunk,
                       max_num_batched_tokens=max_batched)
    runner = ModelRunner(num_blocks=num_blocks)
    eng = LLMEngine(cfg, runner=runner)
    res = {}

    def add(i):
        prompt = [11 + 5 * i + j for j in range(3 + 2 * i + (i % 3) * 9)]
        sp = SamplingParams(temperature=0.0, max_tokens=6 + 4 * (i % 9), stop_token_ids=[EOS])
        eng.add_request(f"r{i}", prompt, sp,
                        on_output=lambda o, i=i: res.setdefault(i, []).extend(o.token_ids))

    for i in range(n_req):
        add(i)
    k, step = n_req, 0
    while eng.has_work() or k < n_req + late:
        if k < n_req + late and step % 3 == 2:   # a late prompt every third step
            add(k)
            k += 1
        eng.step()
        step += 1
    os.environ.pop("ENGINE_PIPELINE_SHRINK", None)
    os.environ.pop("ENGINE_MIXED_AHEAD", None)
    os.environ.pop("ENGINE_MIXED_CHAIN", None)
    assert eng.bm.num_free() == eng.bm.num_blocks
    assert all(q.inflight == 0 and q.pf_sched == 0 for q in eng.scheduler.by_id.values())
    return [res.get(i, []) for i in range(n_req + late)], eng, runner


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_pipelined_decode_with_finishes_matches_synchronous(depth):
    ref, _, _ = _run(False, 1)
    got, eng, runner = _run(True, depth)
    assert got == ref
    # sequences of different lengths stop mid-pipeline: the queue shrank instead of
    # draining, and every shrunk step gathered its ids by row map
    assert eng.stats["pipeline_shrinks"] > 0
    assert any(rm is not None for _, _, rm in runner.launches)
    lens = sorted({len(o) for o in ref})
    assert len(lens) > 2   # the finishes really are staggered


def test_shrink_keeps_pipelining_until_last_sequence():
    """With every request admitted up front, the only synchronous (non-queued)
    launch is the first decode step: later stops shrink the queue."""
    _, eng, runner = _run(True, 1)
    first_launches = [l for l in runner.launches if l[1] == 0]
    assert len(first_launches) == 1


def test_default_drains_on_stop():
    """Default (ENGINE_PIPELINE_SHRINK unset): a stop drains the queue, so the
    session's next prompt is scheduled one step sooner; tokens are unchanged."""
    ref, _, _ = _run(False, 1, shrink=False)
    got, eng, runner = _run(True, 1, shrink=False)
    assert got == ref
    assert eng.stats["pipeline_shrinks"] == 0
    assert all(rm is None for _, _, rm in runner.launches)


@pytest.mark.parametrize("depth", [1, 2])
def test_mixed_ahead_matches_synchronous(depth):
    """Prompts that arrive while decode steps are queued are scheduled into a mixed
    step queued behind them (decode rows' ids gathered by row map from the last
    queued step); tokens equal the synchronous engine's, every block comes back."""
    ref, _, _ = _run(False, 1, n_req=4, late=14)
    got, eng, runner = _run(True, depth, n_req=4, late=14, mixed_ahead=True)
    assert got == ref
    assert eng.stats["mixed_ahead"] > 0 and runner.mixed
    # decode steps were queued behind mixed ones (ids from the mixed step's rows)
    assert eng.stats["pipelined_steps"] > 0
    # without the chain the drained path ran the rest synchronously: every queued
    # mixed step sat behind a decode step
    assert all(d > 0 and rm is not None for d, _, rm in runner.mixed)


@pytest.mark.parametrize("depth", [1, 2])
@pytest.mark.parametrize("budget", [8192, 20])
def test_mixed_chain_matches_synchronous(depth, budget):
    """Mixed chain: a drained queue launches its mixed step (ids from the host) and
    further mixed steps queue behind running ones, continuing chunked prompts after
    their queued chunks (``budget`` 20 tokens per step: long prompts are split over
    several chained steps).  Tokens equal the synchronous engine's, chunks are
    contiguous, every block comes back and no chunk stays counted as scheduled."""
    ref, _, _ = _run(False, 1, n_req=6, late=12, max_batched=budget)
    got, eng, runner = _run(True, depth, n_req=6, late=12, mixed_ahead=True, chain=True,
                            max_batched=budget)
    assert got == ref
    assert eng.stats["mixed_drained_launch"] > 0
    assert any(rm is None for _, _, rm in runner.mixed)
    if budget == 20:
        assert eng.stats["mixed_chain"] > 0
        # rows that joined after the last queued step was built take their host id
        assert any(rm and min(rm) < 0 for _, _, rm in runner.mixed)


@pytest.mark.parametrize("depth", [1, 2])
def test_mixed_chain_under_kv_pressure(depth):
    """chained prefill chunks whose sequence is reset while they are in
    flight (recompute preemption under a tiny KV pool: ``_reset_to_waiting`` drops the
    blocks and bumps the epoch).  The queued chunk is ignored by its post_step, the
    prompt re-prefills from the start, tokens still equal the synchronous engine's,
    every block comes back and nothing stays counted as scheduled or in flight."""
    ref, eng0, _ = _run(False, 1, n_req=6, late=12, max_batched=20, num_blocks=40)
    got, eng, runner = _run(True, depth, n_req=6, late=12, mixed_ahead=True, chain=True,
                            max_batched=20, num_blocks=40)
    assert got == ref
    assert eng.scheduler.num_preemptions > 0      # the pool really ran out mid-chain
    assert eng.scheduler.stale_chunks > 0         # ... and dropped chunks still in flight
    assert eng.stats["mixed_chain"] > 0


def test_mixed_ahead_with_background_warmups():
    """Background prefix-cache warm-ups queued while decode steps run are prefilled
    in mixed steps queued ahead too; foreground tokens are unchanged and every
    block comes back (warm-up blocks stay cached, not held)."""
    import os

    outs = []
    for ahead in (False, True):
        os.environ["ENGINE_MIXED_AHEAD"] = "1" if ahead else "0"
        cfg = EngineConfig(model="tiny", device="cpu", block_size=4, async_output=ahead,
                           pipeline_depth=1, max_num_seqs=32)
        runner = ModelRunner()
        eng = LLMEngine(cfg, runner=runner)
        res = {}
        for i in range(5):
            eng.add_request(f"r{i}", [7 + i + j for j in range(5 + 3 * i)],
                            SamplingParams(temperature=0.0, max_tokens=20 + i, stop_token_ids=[EOS]),
                            on_output=lambda o, i=i: res.setdefault(i, []).extend(o.token_ids))
        step = 0
        while eng.has_work():
            if step in (3, 6, 9):
                eng.add_request(f"w{step}", [300 + step + j for j in range(30)],
                                SamplingParams(temperature=0.0, max_tokens=1), background=True)
            eng.step()
            step += 1
        os.environ.pop("ENGINE_MIXED_AHEAD", None)
        assert eng.bm.num_free() == eng.bm.num_blocks
        outs.append([res.get(i, []) for i in range(5)])
        if ahead:
            assert eng.stats["mixed_ahead"] > 0
    assert outs[0] == outs[1]


def _slow_step_done(self, h) -> bool:
    """step_done() is False for the first two polls of every queued step."""
    polls = self.__dict__.setdefault("polls", {})
    n = polls.get(id(h), 0)
    polls[id(h)] = n + 1
    return n >= 2


# named ModelRunner too: the engine pipelines only ``ModelRunner``s
_SlowDone = type("ModelRunner", (ModelRunner,), {"step_done": _slow_step_done})


def test_prompt_arriving_during_drain_is_queued_behind_running_step():
    """A stop drains the queue; a prompt admitted while the last queued step still
    runs (AsyncEngine's poll hook) goes into a mixed step queued behind it.
    Tokens equal the synchronous engine's; blocks all come back."""
    import os

    def run(async_output):
        os.environ["ENGINE_MIXED_AHEAD"] = "1"
        cfg = EngineConfig(model="tiny", device="cpu", block_size=4, async_output=async_output,
                           pipeline_depth=1, max_num_seqs=32)
        runner = _SlowDone()
        eng = LLMEngine(cfg, runner=runner)
        res = {}
        pending = []

        def add(i):
            eng.add_request(f"r{i}", [9 + 3 * i + j for j in range(4 + 5 * (i % 4))],
                            SamplingParams(temperature=0.0, max_tokens=5 + 3 * (i % 5),
                                           stop_token_ids=[EOS]),
                            on_output=lambda o, i=i: res.setdefault(i, []).extend(o.token_ids))

        def poll():   # the next request "arrives" while a step runs
            if pending:
                add(pending.pop(0))

        eng.poll_hook = poll if async_output else None
        for i in range(4):
            add(i)
        nxt, step = 4, 0
        while eng.has_work() or pending or nxt < 16:
            if nxt < 16 and not pending and step % 3 == 0:
                pending.append(nxt)
                nxt += 1
            if not async_output or not eng.has_work():
                poll()   # between steps (AsyncEngine drains its command queue there too)
            eng.step()
            step += 1
        os.environ.pop("ENGINE_MIXED_AHEAD", None)
        assert eng.bm.num_free() == eng.bm.num_blocks
        return [res.get(i, []) for i in range(16)], eng

    ref, _ = run(False)
    got, eng = run(True)
    assert got == ref
    assert eng.stats["mixed_ahead_drain"] > 0


def _failing_collect(self, h):
    """decode_collect fails once a mixed step has been queued behind the step (one
    launched from a drained queue, rowmap None, does not count)."""
    if any(rm is not None for _, _, rm in self.mixed) and not self.__dict__.get("failed"):
        self.failed = True
        raise RuntimeError("injected device error")
    return list(h.out)


_FailBehindMixed = type("ModelRunner", (ModelRunner,), {"decode_collect": _failing_collect})


def test_failure_with_a_queued_mixed_step_finishes_every_request():
    """a step that fails while a mixed-ahead step is queued behind it.
    The mixed step's prompts had left `waiting` and would only join `running` in
    post_step; fail_unfinished must end them too (an error output each) and every
    KV block must come back."""
    import os

    os.environ["ENGINE_MIXED_AHEAD"] = "1"
    try:
        cfg = EngineConfig(model="tiny", device="cpu", block_size=4, async_output=True,
                           pipeline_depth=1, max_num_seqs=32)
        runner = _FailBehindMixed()
        eng = LLMEngine(cfg, runner=runner)
        done = {}

        def add(i):
            eng.add_request(f"r{i}", [5 + 2 * i + j for j in range(6 + 3 * i)],
                            SamplingParams(temperature=0.0, max_tokens=40),
                            on_output=lambda o, i=i: done.__setitem__(i, o) if o.finished else None)

        for i in range(3):
            add(i)
        err = None
        for step in range(60):
            if step == 4:
                add(3)
                add(4)
            try:
                eng.step()
            except RuntimeError as e:
                err = e
                break
        assert err is not None and runner.mixed, "the failure must hit with a mixed step queued"
        eng.fail_unfinished(str(err))
    finally:
        os.environ.pop("ENGINE_MIXED_AHEAD", None)
    assert sorted(done) == [0, 1, 2, 3, 4]
    assert all(o.finish_reason == "error" for o in done.values())
    assert not eng.has_work()
    assert eng.bm.num_free() == eng.bm.num_blocks


# ---- pipelined guided decoding (deferred sampler) --------------------------------

def _pick(tok: int, pos: int, mask_row) -> int:
    """The fake model's sample under an allow-mask row: unguided rows (all ones)
    follow _next; guided rows pick deterministically among the allowed ids."""
    import numpy as np

    if mask_row is None or (mask_row == -1).all():
        return _next(tok, pos)
    allowed = np.nonzero(np.unpackbits(mask_row.view(np.uint8), bitorder="little"))[0]
    assert len(allowed), "an empty allow-mask row"
    return int(allowed[(tok * 131 + pos * 7) % len(allowed)])


class _GHandle(_Handle):
    def __init__(self, ids, pos, pending):
        super().__init__(None)
        self.ids, self.pos, self.pending = ids, pos, pending


class _GuidedRunner(ModelRunner):
    """Emulates the split decode graphs: a deferred launch runs the 'forward'
    (fixes input ids and positions) and leaves the sample to sample_launch, which
    gets the masks the engine computes from the previous step's tokens."""

    def can_defer_sample(self) -> bool:
        return True

    def execute(self, batch, masks):
        self.stats["steps"] += 1
        return [_pick(int(s.tokens[-1]), s.n_tokens - 1, None if masks is None else masks[i])
                for i, s in enumerate(batch.sampled_seqs())]

    def decode_launch(self, seqs, ahead=0, masks=None, rowmap=None, defer_sample=False):
        self.launches.append((len(seqs), ahead, None if rowmap is None else list(rowmap)))
        if ahead:
            rows = rowmap if rowmap is not None else range(len(seqs))
            ids = [self.d_out[r] for r in rows]
        else:
            ids = [int(s.tokens[-1]) for s in seqs]
        pos = [s.n_tokens - 1 + s.inflight for s in seqs]
        for s, p in zip(seqs, pos):
            assert p // self.bs < len(s.block_ids), "KV slot of a queued step has no block"
        h = _GHandle(ids, pos, defer_sample)
        if defer_sample:
            self.d_out = None   # the next step may not read ids that are not sampled yet
            self.stats["deferred"] = self.stats.get("deferred", 0) + 1
        else:
            self._sample(h, masks)
        return h

    def _sample(self, h, masks):
        h.out = [_pick(t, p, None if masks is None else masks[i])
                 for i, (t, p) in enumerate(zip(h.ids, h.pos))]
        self.d_out = h.out
        h.pending = False

    def sample_launch(self, h, masks):
        assert h.pending
        self._sample(h, masks)

    def decode_collect(self, h):
        assert not h.pending, "collected a step whose sampler never ran"
        return list(h.out)

    def mixed_launch(self, batch, rowmap, masks=None, defer_sample=False):
        """Mixed step: decode rows' ids from the last queued step (rowmap) or the host
        (None / -1), completed prompts sample at their last position; a deferred
        sampler waits for sample_launch (guided rows behind a queued step)."""
        self.mixed.append((len(batch.decode_seqs), list(batch.prefill_tokens),
                           None if rowmap is None else list(rowmap)))
        ids, pos = [], []
        for i, s in enumerate(batch.decode_seqs):
            if rowmap is None or rowmap[i] < 0:
                assert s.inflight == 0
                ids.append(int(s.tokens[-1]))
            else:
                assert s.inflight >= 1 and self.d_out is not None
                ids.append(self.d_out[rowmap[i]])
            pos.append(s.n_tokens - 1 + s.inflight)
            assert pos[-1] // self.bs < len(s.block_ids)
        starts = batch.prefill_start or [s.num_computed for s in batch.prefill_seqs]
        for s, n, smp, a in zip(batch.prefill_seqs, batch.prefill_tokens, batch.prefill_sample, starts):
            assert (a + n + self.bs - 1) // self.bs <= len(s.block_ids)
            if smp:
                assert a + n == s.n_tokens
                ids.append(int(s.tokens[-1]))
                pos.append(s.n_tokens - 1)
        h = _GHandle(ids, pos, defer_sample)
        if defer_sample:
            self.d_out = None
            self.stats["deferred_mixed"] = self.stats.get("deferred_mixed", 0) + 1
        else:
            self._sample(h, masks)
        return h

    def mixed_collect(self, h):
        assert not h.pending, "collected a mixed step whose sampler never ran"
        return list(h.out)

_GuidedRunner.__name__ = "ModelRunner"


def test_guided_batches_pipeline_with_deferred_sampler():
    """Guided (tool-call grammar) and free sequences decode together pipelined: the
    step behind the running one is queued without its sampler, which goes in once
    the running step's tokens moved the grammars.  Tokens equal the synchronous
    engine's; forced runs (jump-forward) drop the queued sample and drain."""
    import json
    import os

    from fasttalk_llm_microservice_amd.engine.guided import GuidedSpec, tool_call_ast

    tools = [{"type": "function", "function": {"name": "duckduckgo_search", "parameters": {
        "type": "object", "properties": {"query": {"type": "string", "maxLength": 24},
                                         "max_results": {"type": "integer"}},
        "required": ["query", "max_results"]}}}]
    spec = GuidedSpec(tool_call_ast(tools))

    def run(async_output):
        os.environ["ENGINE_MIXED_AHEAD"] = "0"
        cfg = EngineConfig(model="tiny", device="cpu", block_size=4, async_output=async_output,
                           pipeline_depth=1, max_num_seqs=32)
        runner = _GuidedRunner()
        eng = LLMEngine(cfg, runner=runner)
        res = {}
        for i in range(6):
            guided = i % 2 == 0
            sp = SamplingParams(temperature=0.0, max_tokens=60 if guided else 10 + 3 * i,
                                stop_token_ids=None if guided else [EOS],
                                guided=spec if guided else None)
            eng.add_request(f"r{i}", [20 + 3 * i + j for j in range(4 + i)], sp,
                            on_output=lambda o, i=i: res.setdefault(i, []).extend(o.token_ids))
        while eng.has_work():
            eng.step()
        os.environ.pop("ENGINE_MIXED_AHEAD", None)
        assert eng.bm.num_free() == eng.bm.num_blocks
        assert all(q.inflight == 0 and q.drop_next == 0 for q in eng.scheduler.by_id.values())
        return [res.get(i, []) for i in range(6)], eng, runner

    ref, _, _ = run(False)
    got, eng, runner = run(True)
    assert got == ref
    for i in (0, 2, 4):   # the guided ones are valid calls
        call = json.loads(eng.tokenizer.decode(got[i]))
        assert call["name"] == "duckduckgo_search"
    assert eng.stats["guided_pipelined_steps"] > 0 and runner.stats.get("deferred", 0) > 0
    assert eng.stats["jump_forward_tokens"] > 0 and eng.stats["pipelined_jump_drops"] > 0



def test_guided_rows_chain_mixed_steps_with_deferred_sampler():
    """Mixed chain with guided rows: prompts arriving while guided tool calls decode
    are prefilled in mixed steps queued behind them, whose sampler waits for the
    guided rows' masks (ENGINE_MIXED_CHAIN_GUIDED).  Tokens equal the synchronous
    engine's; every block and in-flight count comes back."""
    import json
    import os

    from fasttalk_llm_microservice_amd.engine.guided import GuidedSpec, tool_call_ast

    tools = [{"type": "function", "function": {"name": "duckduckgo_search", "parameters": {
        "type": "object", "properties": {"query": {"type": "string", "maxLength": 24},
                                         "max_results": {"type": "integer"}},
        "required": ["query", "max_results"]}}}]
    spec = GuidedSpec(tool_call_ast(tools))

    def run(async_output):
        os.environ["ENGINE_MIXED_AHEAD"] = "1"
        os.environ["ENGINE_MIXED_CHAIN"] = "1"
        cfg = EngineConfig(model="tiny", device="cpu", block_size=4, async_output=async_output,
                           pipeline_depth=1, max_num_seqs=32, max_num_batched_tokens=24)
        runner = _GuidedRunner()
        eng = LLMEngine(cfg, runner=runner)
        res = {}

        def add(i):
            guided = i % 3 == 0
            sp = SamplingParams(temperature=0.0, max_tokens=60 if guided else 8 + 3 * (i % 4),
                                stop_token_ids=None if guided else [EOS],
                                guided=spec if guided else None)
            eng.add_request(f"r{i}", [20 + 3 * i + j for j in range(5 + (i % 5) * 4)], sp,
                            on_output=lambda o, i=i: res.setdefault(i, []).extend(o.token_ids))

        for i in range(4):
            add(i)
        k, step = 4, 0
        while eng.has_work() or k < 14:
            if k < 14 and step % 2 == 1:
                add(k)
                k += 1
            eng.step()
            step += 1
        for v in ("ENGINE_MIXED_AHEAD", "ENGINE_MIXED_CHAIN"):
            os.environ.pop(v, None)
        assert eng.bm.num_free() == eng.bm.num_blocks
        assert all(q.inflight == 0 and q.drop_next == 0 and q.pf_sched == 0
                   for q in eng.scheduler.by_id.values())
        return [res.get(i, []) for i in range(14)], eng, runner

    ref, _, _ = run(False)
    got, eng, runner = run(True)
    assert got == ref
    for i in range(0, 14, 3):   # the guided ones are valid calls
        assert json.loads(eng.tokenizer.decode(got[i]))["name"] == "duckduckgo_search"
    assert eng.stats["mixed_deferred_sample"] > 0 and eng.stats["guided_pipelined_mixed"] > 0
