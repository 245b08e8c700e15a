"""Tensor parallelism on the CPU over gloo (SURVEY.md §4 "Distributed": TP logic
runs with 2 processes, no GPU).  Rank 0 is this test process; rank 1 is a
spawned worker fed by the shared-memory step broadcast.  Weights of small
models are drawn unsharded from one seed and sliced, so TP=2 must reproduce
TP=1 token for token."""
import multiprocessing as mp
import time

import numpy as np
import pytest

from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import LLMEngine
from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams
from fasttalk_llm_microservice_amd.parallel.shm_broadcast import ShmBroadcast


def _cfg(**kw):
    base = dict(model="tiny", device="cpu", num_kv_blocks=256, max_model_len=1024, max_num_seqs=8,
                max_num_batched_tokens=64)
    base.update(kw)
    return EngineConfig(**base)


@pytest.mark.parametrize("tp", [2, 4])
def test_tp_generation_matches_tp1(tp):
    """TP=4 splits tiny's 2 kv heads over 4 ranks: each kv head is replicated on two
    ranks (weights.kv_head_range) and the step ring has 3 readers."""
    from fasttalk_llm_microservice_amd.parallel.tp import spawn_tp_engine

    rng = np.random.default_rng(0)
    prompts = [rng.integers(0, 120000, n).tolist() for n in (9, 70, 30)]
    sp = SamplingParams(temperature=0, max_tokens=6, ignore_eos=True)
    ref = LLMEngine(_cfg()).generate(prompts, sp)
    eng = spawn_tp_engine(_cfg(tp_size=tp))
    try:
        assert eng.runner.model.nq == 8 // tp and eng.runner.model.nkv == 1  # heads per rank
        assert len(eng.tp_group.procs) == tp - 1
        out = eng.generate(prompts, sp)
        # seeded sampling is identical across ranks too (every rank samples the gathered logits)
        sp2 = SamplingParams(temperature=0.8, top_p=0.9, max_tokens=4, seed=7, ignore_eos=True)
        out2 = eng.generate(prompts[:1], sp2)
    finally:
        eng.shutdown()
    assert out == ref
    assert out2 == LLMEngine(_cfg()).generate(prompts[:1], sp2)


def test_tp2_fp8_kv_matches_tp1():
    """fp8 KV caches under TP: each rank stores its kv heads in e4m3 and the tokens
    match the single-rank fp8 engine."""
    from fasttalk_llm_microservice_amd.parallel.tp import spawn_tp_engine

    rng = np.random.default_rng(1)
    prompts = [rng.integers(0, 120000, n).tolist() for n in (12, 40)]
    sp = SamplingParams(temperature=0, max_tokens=6, ignore_eos=True)
    ref = LLMEngine(_cfg(kv_cache_dtype="fp8")).generate(prompts, sp)
    eng = spawn_tp_engine(_cfg(tp_size=2, kv_cache_dtype="fp8"))
    try:
        assert str(eng.runner.kv[0][0].dtype) == "torch.float8_e4m3fn"
        out = eng.generate(prompts, sp)
    finally:
        eng.shutdown()
    assert out == ref


def _reader(name, idx, q):
    b = ShmBroadcast(2, name=name, create=False, reader_index=idx, num_slots=4, slot_bytes=1 << 12)
    total = 0
    while True:
        m = b.recv(timeout=30)
        if m is None:
            break
        total += int(m["x"].sum())
    q.put(total)
    b.close()


def test_shm_broadcast_ring_and_overflow():
    w = ShmBroadcast(2, num_slots=4, slot_bytes=1 << 12)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_reader, args=(w.name, i, q)) for i in range(2)]
    for p in ps:
        p.start()
    expect = 0
    for i in range(200):
        x = np.arange(i % 7 * 300 + 1)  # every 7th message overflows the 4 KiB slot
        expect += int(x.sum())
        w.send({"x": x}, timeout=30)
    w.send(None, timeout=30)
    got = sorted([q.get(timeout=60), q.get(timeout=60)])
    for p in ps:
        p.join(timeout=30)
    w.close()
    assert got == [expect, expect]


def test_dp2_router_session_affinity_and_outputs():
    import asyncio

    from fasttalk_llm_microservice_amd.parallel.dp_router import MultiGPUEngine

    rng = np.random.default_rng(3)
    prompts = [rng.integers(0, 120000, n).tolist() for n in (12, 40, 25, 7)]
    sp = SamplingParams(temperature=0, max_tokens=5, ignore_eos=True)
    ref = LLMEngine(_cfg()).generate(prompts, sp)
    eng = MultiGPUEngine(_cfg(dp_size=2)).start()
    try:
        async def one(i, p, sid):
            ids = []
            async for o in eng.generate(p, sp, request_id=f"{sid}#{i}"):
                ids.extend(o.token_ids)
            return ids

        async def run():
            return await asyncio.gather(*[one(i, p, f"sess{i % 2}") for i, p in enumerate(prompts)])

        out = asyncio.run(run())
        assert out == ref
        # each conversation stayed on one replica, and both replicas were used
        assert set(eng._affinity) == {"sess0", "sess1"}
        assert len(set(eng._affinity.values())) == 2
        assert eng.is_healthy() and eng.model_info()["data_parallel_size"] == 2
        time.sleep(0.6)
        asyncio.run(one(9, prompts[0], "sess0"))
        assert eng.engine.metrics()["replicas"] == 2
        # a background warm-up reaches the replica that owns the session,
        # so that session's next turn re-attaches the warmed prefix
        warm = rng.integers(0, 120000, 96).tolist()
        eng.prefill_background(warm, session_id="sess1")
        time.sleep(1.5)

        async def cached(sid):
            n = 0
            async for o in eng.generate(warm + [5, 6, 7], sp, request_id=f"{sid}#w"):
                n = max(n, o.num_cached_tokens)
            return n
        assert asyncio.run(cached("sess1")) >= 64
    finally:
        eng.shutdown()


def test_tp_worker_death_turns_health_red():
    """SURVEY §5 "TP worker death -> health 503": AsyncEngine.is_healthy consults
    TPGroup.alive(), so /health flips as soon as a worker process is gone (rank 0
    may be blocked in a collective that never completes)."""
    from fasttalk_llm_microservice_amd.engine.engine import AsyncEngine
    from fasttalk_llm_microservice_amd.parallel.shm_broadcast import PeerDied
    from fasttalk_llm_microservice_amd.parallel.tp import spawn_tp_engine

    eng = spawn_tp_engine(_cfg(tp_size=2))
    ae = AsyncEngine(eng).start()
    try:
        assert ae.is_healthy()
        worker = eng.tp_group.procs[0]
        worker.kill()
        worker.join(timeout=30)
        assert not ae.is_healthy()
        # a dead peer is fatal for the group (not a per-request failure)
        assert not AsyncEngine._recoverable(PeerDied("x"))
    finally:
        ae._stop = True
        ae._wake.set()
        eng.tp_group.bcast.liveness = lambda: False  # shutdown must not wait for the dead worker
        eng.shutdown()


def test_separate_process_tp_engine_restarts_after_worker_death(monkeypatch):
    """A TP group in its own process (the default for tp_size > 1): when a worker
    dies the replica reports itself dead and exits, the router is unhealthy, fails
    the replica's requests, respawns the group in a fresh process and serves the
    same tokens again."""
    import asyncio

    import psutil

    from fasttalk_llm_microservice_amd.parallel.dp_router import MultiGPUEngine

    monkeypatch.setenv("ENGINE_RESTART_DELAY", "0.2")
    rng = np.random.default_rng(5)
    prompts = [rng.integers(0, 120000, n).tolist() for n in (12, 31)]
    sp = SamplingParams(temperature=0, max_tokens=5, ignore_eos=True)
    ref = LLMEngine(_cfg()).generate(prompts, sp)
    cfg = _cfg(tp_size=2)
    assert cfg.separate_process is False  # dataclass default; from_env defaults TP to True
    from fasttalk_llm_microservice_amd.engine.config import EngineConfig

    monkeypatch.setenv("ENGINE_TP_SIZE", "2")
    assert EngineConfig.from_env(model="tiny").separate_process is True
    eng = MultiGPUEngine(cfg).start()

    async def one(p, rid):
        ids = []
        async for o in eng.generate(p, sp, request_id=rid):
            ids.extend(o.token_ids)
        return ids

    try:
        assert asyncio.run(one(prompts[0], "a#0")) == ref[0]
        rep = eng.replicas[0]
        kids = [c for c in psutil.Process(rep.proc.pid).children()
                if "resource_tracker" not in " ".join(c.cmdline())]
        assert kids, "the replica must own its TP worker process"
        for c in kids:
            c.kill()
        t0 = time.time()
        while eng.is_healthy() and time.time() - t0 < 30:
            time.sleep(0.1)
        assert not eng.is_healthy(), "a dead TP worker must make the engine unhealthy"
        while not eng.is_healthy() and time.time() - t0 < 240:
            time.sleep(0.2)
        assert eng.is_healthy() and eng.restarts == 1 and eng.replicas[0] is not rep
        assert asyncio.run(one(prompts[1], "b#0")) == ref[1]
    finally:
        eng.shutdown()
