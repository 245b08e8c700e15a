"""bench.py --gpus N starts N ranks itself (VERDICT r2 "next" #1): the launcher
path runs before torch is imported, the ranks rendezvous on 127.0.0.1, rank 0
prints ONE JSON line with ``ranks == N`` and the distinct-device count as
``n_gpus`` (0 on the CPU backend).  Run on the CPU over gloo with the tiny model."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _run(args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=timeout)


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{\"metric\"")]


@pytest.mark.parametrize("mode", ["dp", "tp"])
def test_gpus_flag_launches_ranks(mode):
    extra = ["--tp", "2"] if mode == "tp" else []
    r = _run(["--gpus", "2", "--device", "cpu", "--model", "tiny", "--sessions", "2", "--steps", "1",
              "--warmup", "1", "--gen", "4", "--words", "6"] + extra)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    out = lines[0]
    assert out["ranks"] == 2 and out["n_gpus"] == 0 and out["device"] == "cpu"
    assert out["steps"] == 1 and out["warmup"] == 1 and out["value"] > 0
    assert out["config"]["parallelism"] == ("tp2" if mode == "tp" else "dp2")
    if mode == "dp":
        assert out["config"]["global_batch"] == 4  # weak scaling: sessions per rank
        # default DP topology: the shipping front door placed 2 sessions on each worker
        assert out["serve"]["sessions_per_worker"] == [2, 2], out["serve"]
    assert out["config"]["ctx_mean"] and out["config"]["ctx_max"] >= out["config"]["ctx_mean"]


def test_world_size_mismatch_is_refused():
    r = _run(["--gpus", "4", "--device", "cpu", "--model", "tiny"],
             env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


def test_missing_gpus_fail_loudly():
    """Two ranks on the GPU path with fewer visible GPUs than ranks: every rank
    exits non-zero (no silent one-GPU run labelled as two)."""
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--sessions", "1"],
             env_extra={"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": ""}, timeout=180)
    assert r.returncode != 0
    assert not _json_lines(r.stdout)


def test_eight_ranks_through_the_front_door():
    """the 8-rank data-parallel path of ``bench.py --gpus 8`` end to
    end on the CPU (gloo): 8 ranks, the shipping front door spreading the 24 sessions
    evenly (spread <= 1), and the record names its backend, world size and every
    rank's device placement."""
    r = _run(["--gpus", "8", "--device", "cpu", "--model", "tiny", "--serve", "door",
              "--sessions", "3", "--steps", "1", "--warmup", "1", "--gen", "4", "--words", "6"],
             timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    out = lines[0]
    assert out["ranks"] == 8 and out["world_size"] == 8 and out["dist_backend"] == "gloo"
    assert out["config"]["parallelism"] == "dp8" and out["config"]["global_batch"] == 24
    spw = out["serve"]["sessions_per_worker"]
    assert len(spw) == 8 and sum(spw) == 24 and max(spw) - min(spw) <= 1, spw
    assert sorted(d["rank"] for d in out["rank_devices"]) == list(range(8))


def test_fp8_kv_cache_flag_reaches_the_engine_and_the_json():
    """--kv-cache-dtype fp8 sets ENGINE_KV_CACHE_DTYPE for the service the bench drives
    (one rank here), the run completes on the fp8 pool and the JSON line says so."""
    r = _run(["--device", "cpu", "--model", "tiny", "--sessions", "2", "--steps", "1", "--warmup", "1",
              "--gen", "4", "--words", "6", "--kv-cache-dtype", "fp8"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json_lines(r.stdout)[0]
    assert out["kv_cache_dtype"] == "fp8 (e4m3)" and out["value"] > 0
