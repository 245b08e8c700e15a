"""Failure detection and tracing hooks: an injected step failure
fails only the in-flight requests and the engine keeps serving; a fatal one
(MemoryError, a sticky HIP fault, or a streak of failing steps) turns /health
unhealthy; FT_PROFILE writes a torch.profiler trace."""
import asyncio
import glob
import os

import pytest

from fasttalk_llm_microservice_amd.engine.config import EngineConfig
from fasttalk_llm_microservice_amd.engine.engine import AsyncEngine, EngineError, LLMEngine
from fasttalk_llm_microservice_amd.engine.sampling_params import SamplingParams


def _async_engine():
    return AsyncEngine(LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=128,
                                              max_model_len=512, max_num_seqs=4))).start()


async def _collect(eng, prompt, n):
    outs = []
    async for o in eng.generate(prompt, SamplingParams(temperature=0, max_tokens=n, ignore_eos=True)):
        outs.append(o)
    return outs


def test_recoverable_step_failure(monkeypatch):
    monkeypatch.setenv("FT_FAULT_STEP", "3")
    monkeypatch.setenv("FT_FAULT_KIND", "runtime")
    eng = _async_engine()
    try:
        first = asyncio.run(_collect(eng, [1, 2, 3], 20))
        assert first[-1].finished and first[-1].finish_reason == "error"
        assert "FT_FAULT" in first[-1].error
        again = asyncio.run(_collect(eng, [4, 5, 6], 5))
        assert again[-1].finish_reason == "length" and sum(len(o.token_ids) for o in again) == 5
        assert eng.is_healthy()
        assert eng.engine.bm.num_free() == eng.engine.bm.num_blocks
    finally:
        eng.shutdown()


def test_fatal_step_failure_marks_unhealthy(monkeypatch):
    monkeypatch.setenv("FT_FAULT_STEP", "2")
    monkeypatch.setenv("FT_FAULT_KIND", "oom")
    eng = _async_engine()
    try:
        out = asyncio.run(_collect(eng, [1, 2, 3], 10))
        assert out[-1].finish_reason == "error"
        assert not eng.is_healthy()
        with pytest.raises(EngineError):
            asyncio.run(_collect(eng, [1], 2))
    finally:
        eng.shutdown()


def test_profiler_trace(monkeypatch, tmp_path):
    monkeypatch.setenv("FT_PROFILE", "2")
    monkeypatch.setenv("FT_PROFILE_SKIP", "1")
    monkeypatch.setenv("FT_PROFILE_DIR", str(tmp_path))
    eng = LLMEngine(EngineConfig(model="tiny", device="cpu", num_kv_blocks=64, max_model_len=256))
    eng.generate([[1, 2, 3]], SamplingParams(temperature=0, max_tokens=5, ignore_eos=True))
    traces = glob.glob(os.path.join(tmp_path, "engine_steps_*.json"))
    assert traces and os.path.getsize(traces[0]) > 0


@pytest.mark.parametrize("kind,repeat", [("device", 1), ("runtime", 3)])
def test_device_fault_or_failure_streak_marks_unhealthy(monkeypatch, kind, repeat):
    monkeypatch.setenv("FT_FAULT_STEP", "2")
    monkeypatch.setenv("FT_FAULT_KIND", kind)
    monkeypatch.setenv("FT_FAULT_REPEAT", str(repeat))
    eng = _async_engine()
    try:
        for _ in range(repeat):
            out = asyncio.run(_collect(eng, [1, 2, 3], 10))
            assert out[-1].finish_reason == "error"
        assert not eng.is_healthy()
        assert eng.engine.bm.num_free() == eng.engine.bm.num_blocks
    finally:
        eng.shutdown()


def test_failure_streak_resets_after_a_good_step(monkeypatch):
    monkeypatch.setenv("FT_FAULT_STEP", "2")
    monkeypatch.setenv("FT_FAULT_REPEAT", "2")
    eng = _async_engine()
    try:
        for _ in range(2):
            assert asyncio.run(_collect(eng, [1, 2, 3], 10))[-1].finish_reason == "error"
        assert eng.is_healthy()
        assert asyncio.run(_collect(eng, [4, 5], 4))[-1].finish_reason == "length"
        assert eng._fail_streak == 0 and eng.is_healthy()
    finally:
        eng.shutdown()


def test_classifies_device_oom_as_fatal():
    import torch

    assert not AsyncEngine._recoverable(torch.cuda.OutOfMemoryError("HIP out of memory"))
    assert not AsyncEngine._recoverable(RuntimeError("HIP error: an illegal memory access"))
    assert AsyncEngine._recoverable(ValueError("prompt too long"))
