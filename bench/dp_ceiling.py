"""Single-endpoint DP serving ceiling: ONE service process -- the
real FastAPI ``/ws/llm`` app on the aiohttp ASGI transport, the voice agent,
NativeHandler, the DP router -- in front of N engine replica processes whose
model step is synthetic (``ENGINE_SYNTHETIC_STEP_MS``: sleep for a GPU step's
time, deterministic one-word tokens; scheduler, KV manager, detokenizer and the
replica pipes run for real).  K load-generator processes drive 50 sessions per
replica.  Reports delivered output tok/s against the replicas' ideal rate
(N x 50 / step), TTFT percentiles and the service process's CPU use, i.e.
whether one process can stream what N MI355X replicas produce.

python bench/dp_ceiling.py [--replicas 8] [--step-ms 7.5] [--turns 3] [--gen 128] [--clients 4]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--sessions-per-replica", type=int, default=50)
    ap.add_argument("--step-ms", type=float, default=7.5)
    ap.add_argument("--turns", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--words", type=int, default=40)
    ap.add_argument("--clients", type=int, default=4)
    ap.add_argument("--no-agent", action="store_true")
    ap.add_argument("--port", type=int, default=18950)
    ap.add_argument("--profile", default="", help="cProfile the event-loop thread into this file")
    ap.add_argument("--mode", default="router", choices=["router", "workers"],
                    help="router: one service process + N replica processes (ENGINE_DP_MODE=router); "
                         "workers: N service processes on one port, one engine each")
    a = ap.parse_args()
    env = {"ENGINE_SYNTHETIC_STEP_MS": str(a.step_ms), "ENGINE_DP_SIZE": str(a.replicas),
           "COMPUTE_DEVICE": "cpu", "LLM_PROVIDER": "native", "ENGINE_MODEL": "llama3-8b",
           "ENABLE_PYDANTIC_AI": "false" if a.no_agent else "true", "LOG_LEVEL": "WARNING",
           "LLM_MAX_CONNECTIONS": str(a.replicas * a.sessions_per_replica + 64),
           "ENGINE_MAX_NUM_SEQS": "256", "ENGINE_DP_MODE": a.mode}
    os.environ.update(env)
    from ws_load import client_process

    sessions = a.replicas * a.sessions_per_replica
    url = f"ws://127.0.0.1:{a.port}/ws/llm"
    cfg = {"system_prompt": "You are a helpful voice assistant.", "temperature": 0.7, "top_p": 0.9,
           "max_tokens": a.gen, "ignore_eos": True}
    ctx = mp.get_context("spawn")
    clients = []
    per = [sessions // a.clients + (1 if i < sessions % a.clients else 0) for i in range(a.clients)]
    for i, n in enumerate(per):
        pc, cc = ctx.Pipe()
        p = ctx.Process(target=client_process, args=(cc, url, n, cfg, a.words, 1000 + i), daemon=True)
        p.start()
        clients.append((p, pc))

    import psutil

    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.server.asgi_aiohttp import AiohttpASGIServer
    from app.utils.config import Config

    t0 = time.time()
    if a.mode == "workers":
        return run_workers(a, clients, t0)
    c = Config()
    c.port = a.port
    server = WebSocketLLMServer(c)
    asgi = AiohttpASGIServer(server.app, "127.0.0.1", a.port)
    loop = asyncio.new_event_loop()
    ready = threading.Event()

    prof = None
    if a.profile:
        import cProfile

        prof = cProfile.Profile()

    def serve():
        asyncio.set_event_loop(loop)
        loop.run_until_complete(asgi.start())
        ready.set()
        if prof is not None:
            prof.enable()
        loop.run_forever()
        if prof is not None:
            prof.disable()

    threading.Thread(target=serve, daemon=True).start()
    if not ready.wait(300):
        raise SystemExit("server did not start")
    print(f"service up in {time.time() - t0:.1f}s ({a.replicas} replicas)", flush=True)

    def all_cmd(cmd):
        for _, pc in clients:
            pc.send(cmd)
        res = [pc.recv() for _, pc in clients]
        for r in res:
            if not r.get("ok"):
                raise SystemExit(f"client failed: {r.get('error')}")
        return [r.get("result") for r in res]

    all_cmd("open")
    if a.warmup:
        all_cmd(("run", a.warmup))
    me = psutil.Process(os.getpid())
    me.cpu_percent(None)
    ct0 = me.cpu_times()
    t1 = time.perf_counter()
    res = all_cmd(("run", a.turns))
    dt = time.perf_counter() - t1
    ct1 = me.cpu_times()
    cpu = 100.0 * ((ct1.user - ct0.user) + (ct1.system - ct0.system)) / dt
    all_cmd("close")
    tokens = sum(r["tokens"] for r in res)
    frames = sum(r["frames"] for r in res)
    ttft = sorted(x for r in res for x in r["ttft_s"])
    pct = lambda q: round(1e3 * ttft[min(len(ttft) - 1, int(q * (len(ttft) - 1)))], 1)  # noqa: E731
    ideal = a.replicas * a.sessions_per_replica * 1e3 / a.step_ms
    out = {"mode": "router", "replicas": a.replicas, "sessions": sessions, "step_ms": a.step_ms,
           "path": "agent" if not a.no_agent else "direct",
           "tokens_per_s": round(tokens / dt, 1), "frames_per_s": round(frames / dt, 1),
           "ideal_decode_tokens_per_s": round(ideal, 1),
           "fraction_of_ideal": round(tokens / dt / ideal, 3),
           "p50_ttft_ms": pct(0.5), "p99_ttft_ms": pct(0.99),
           "service_process_cpu_percent": round(cpu, 1), "elapsed_s": round(dt, 2)}
    print(json.dumps(out), flush=True)
    try:
        asyncio.run_coroutine_threadsafe(asgi.stop(), loop).result(timeout=15)
    except Exception:
        pass
    loop.call_soon_threadsafe(loop.stop)
    time.sleep(0.5)
    if prof is not None:
        import pstats

        prof.dump_stats(a.profile)
        pstats.Stats(a.profile).sort_stats("tottime").print_stats(35)
    eng = server.native_handler.engine
    eng.shutdown()


def _cmd(clients, cmd):
    for _, pc in clients:
        pc.send(cmd)
    res = [pc.recv() for _, pc in clients]
    for r in res:
        if not r.get("ok"):
            raise SystemExit(f"client failed: {r.get('error')}")
    return [r.get("result") for r in res]


def run_workers(a, clients, t0):
    """N service worker processes on one port (app/server/workers.py)."""
    import psutil
    import socket

    from app.server.workers import WorkerPool

    pool = WorkerPool(a.replicas, "127.0.0.1", a.port).start()
    try:
        while True:   # every worker listening (connections to a not-yet-ready one would fail)
            time.sleep(1.0)
            if not all(pool.alive()):
                raise SystemExit("a worker died at startup")
            try:
                with socket.create_connection(("127.0.0.1", a.port), timeout=1):
                    pass
            except OSError:
                continue
            time.sleep(max(2.0, 0.5 * a.replicas))
            break
        print(f"{a.replicas} workers up in {time.time() - t0:.1f}s", flush=True)
        _cmd(clients, "open")
        if a.warmup:
            _cmd(clients, ("run", a.warmup))
        procs = [psutil.Process(p.pid) for p in pool.procs]
        ct0 = [p.cpu_times() for p in procs]
        t1 = time.perf_counter()
        res = _cmd(clients, ("run", a.turns))
        dt = time.perf_counter() - t1
        ct1 = [p.cpu_times() for p in procs]
        cpu = [100.0 * ((b.user - x.user) + (b.system - x.system)) / dt for x, b in zip(ct0, ct1)]
        _cmd(clients, "close")
    finally:
        pool.stop()
    tokens = sum(r["tokens"] for r in res)
    frames = sum(r["frames"] for r in res)
    ttft = sorted(x for r in res for x in r["ttft_s"])
    pct = lambda q: round(1e3 * ttft[min(len(ttft) - 1, int(q * (len(ttft) - 1)))], 1)  # noqa: E731
    ideal = a.replicas * a.sessions_per_replica * 1e3 / a.step_ms
    print(json.dumps({"mode": "workers", "replicas": a.replicas,
                      "sessions": a.replicas * a.sessions_per_replica, "step_ms": a.step_ms,
                      "tokens_per_s": round(tokens / dt, 1), "frames_per_s": round(frames / dt, 1),
                      "ideal_decode_tokens_per_s": round(ideal, 1),
                      "fraction_of_ideal": round(tokens / dt / ideal, 3),
                      "p50_ttft_ms": pct(0.5), "p99_ttft_ms": pct(0.99),
                      "worker_cpu_percent": [round(c, 1) for c in cpu], "elapsed_s": round(dt, 2)}),
          flush=True)


if __name__ == "__main__":
    main()
