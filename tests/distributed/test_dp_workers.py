"""DP serving as N service worker processes on one port (app/server/workers.py,
ENGINE_DP_MODE=workers): sessions over SO_REUSEPORT reach every worker, each
streams from its own engine, and a killed worker is restarted and serves again.
CPU only: the engines use the synthetic runner (ENGINE_SYNTHETIC_STEP_MS)."""
import asyncio
import os
import socket
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "bench"))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _wait_listening(port, timeout=120):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            with socket.create_connection(("127.0.0.1", port), timeout=1):
                return
        except OSError:
            time.sleep(0.5)
    raise TimeoutError("workers did not start")


def _sessions(port, n, turns=1, probe=None):
    from ws_load import LoadClient

    cfg = {"system_prompt": "hi", "temperature": 0.0, "max_tokens": 6, "ignore_eos": True}

    async def go():
        lc = LoadClient(f"ws://127.0.0.1:{port}/ws/llm", n, cfg, words=5, seed=1)
        await lc.open()
        try:
            r = await lc.run_turns(turns)
            if probe is not None:
                r["probe"] = probe()
            return r
        finally:
            await lc.close()
    return asyncio.run(go())


def test_dp_workers_share_one_port_and_restart(monkeypatch):
    from app.server.workers import WorkerPool

    for k, v in {"ENGINE_SYNTHETIC_STEP_MS": "2", "COMPUTE_DEVICE": "cpu", "LLM_PROVIDER": "native",
                 "ENGINE_MODEL": "tiny", "ENABLE_PYDANTIC_AI": "false", "LOG_LEVEL": "WARNING"}.items():
        monkeypatch.setenv(k, v)
    port = _free_port()
    pool = WorkerPool(2, "127.0.0.1", port, max_restarts=1).start()
    try:
        _wait_listening(port)
        time.sleep(3)
        import psutil

        def per_worker():   # open sessions each worker holds on the service port
            return [len([c for c in psutil.Process(p.pid).net_connections()
                         if c.status == "ESTABLISHED" and c.laddr and c.laddr.port == port])
                    for p in pool.procs]
        r = _sessions(port, 16, probe=per_worker)
        assert r["turns"] == 16 and r["tokens"] == 16 * 6
        # SO_REUSEPORT spread the connections over both workers
        assert sum(r["probe"]) == 16 and min(r["probe"]) >= 1, r["probe"]
        victim = pool.procs[0]
        victim.kill()
        victim.join(10)
        pool.supervise_once()
        assert pool.restarts[0] == 1 and pool.procs[0] is not victim
        time.sleep(4)
        _wait_listening(port)
        r = _sessions(port, 8)
        assert r["turns"] == 8 and r["tokens"] == 8 * 6
    finally:
        pool.stop()
    assert not any(pool.alive())
