"""Headline benchmark (BASELINE.json): output tokens/sec per node + p50 TTFT over
WebSocket, Llama-3-8B, 50 concurrent sessions with conversation history.

One process per GPU (``torchrun --nproc-per-node N``): every rank serves its own
engine replica (data parallel, weak scaling: 50 sessions per GPU) behind the real
service stack -- FastAPI ``/ws/llm`` on the aiohttp ASGI transport, the
session/conversation managers, the native voice agent (default provider path),
the in-process MI355X engine -- and a load-generator child process drives 50
WebSocket sessions against it.  A *step* is one conversation turn of every
session (user message -> streamed reply of ``--gen`` tokens, ``ignore_eos`` so
every turn has fixed work); history accumulates across warmup and timed turns.

Weights are random-init (no checkpoints offline) with the exact Llama-3-8B
architecture; prompts are synthetic English.

python bench.py [--gpus N] [--steps K] [--warmup W] [--sessions 50] [--gen 128]

``--gpus N`` with N > 1 and no ``WORLD_SIZE`` in the environment: this process
becomes a launcher that starts N rank processes itself (``RANK`` / ``LOCAL_RANK``
/ ``WORLD_SIZE`` / ``MASTER_*`` on 127.0.0.1) before anything touches a GPU, waits
for them and exits with the worst rank's code; rank 0 prints the JSON line.
Under ``torch.distributed.run`` the ranks exist already and ``--gpus`` must equal
``WORLD_SIZE``.  Each rank needs its own GPU unless ``FT_BENCH_SHARED_GPU=1``
(rehearsal: all ranks on the visible GPU(s); the JSON then reports the distinct
devices as ``n_gpus`` and the rank count as ``ranks``).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import signal
import socket
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))


def _p50(xs):
    xs = sorted(xs)
    return round(xs[len(xs) // 2], 2) if xs else None


def _free_port(base: int) -> int:
    for p in range(base, base + 200):
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
                return p
            except OSError:
                continue
    raise RuntimeError("no free port")


def _heartbeat(state: dict, period: float = 30.0):
    """A progress line on stderr every ``period`` s (long TP / multi-rank runs stay
    visibly alive while weights load and graphs capture)."""
    t0 = time.time()

    def run():
        while not state.get("done"):
            time.sleep(period)
            if not state.get("done"):
                print(f"bench: {state.get('phase', '?')} ({time.time() - t0:.0f} s)", file=sys.stderr,
                      flush=True)

    threading.Thread(target=run, daemon=True, name="bench-heartbeat").start()


def _launch_ranks(n: int, argv) -> int:
    """Start ``n`` bench ranks (this file, same arguments) with the torch.distributed
    env contract and wait for them.  Runs before this process imports torch, so it
    never touches a GPU; if one rank fails the others are stopped."""
    env = dict(os.environ)
    shared = env.get("FT_BENCH_SHARED_GPU", "0") == "1"
    if shared and not env.get("ENGINE_GPU_MEMORY_UTILIZATION"):
        # every rank's engine sizes its KV cache from the same device: a 1/n share each,
        # counted against its own allocations only (the others may or may not have sized
        # theirs yet)
        env["ENGINE_GPU_MEMORY_UTILIZATION"] = f"{0.85 / n:.3f}"
        env.setdefault("ENGINE_KV_SIZING", "own")
    port = _free_port(29500 + (os.getpid() % 400))
    procs = []
    for r in range(n):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=e))

    def stop_all(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.time() + 20
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()

    signal.signal(signal.SIGTERM, lambda *_: (stop_all(), sys.exit(143)))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                r = p.poll()
                if r is None:
                    continue
                live.remove(p)
                if r != 0:
                    rc = rc or r
                    print(f"bench launcher: rank {procs.index(p)} exited with {r}; stopping the others",
                          file=sys.stderr, flush=True)
                    stop_all()
                    live = []
                    break
            time.sleep(0.2)
    finally:
        stop_all()
    return rc


def _device_plan(world: int, local_rank: int, device: str):
    """(device index, distinct devices used) for this rank; fails loudly when the
    node has fewer GPUs than ranks, unless FT_BENCH_SHARED_GPU=1."""
    if device != "cuda":
        return None, 0
    import torch

    ndev = torch.cuda.device_count()  # does not initialise the GPU
    if ndev < 1:
        raise SystemExit("bench: no GPU visible")
    if os.environ.get("FT_BENCH_SHARED_GPU", "0") == "1":
        return local_rank % ndev, min(world, ndev)
    if ndev < world:
        raise SystemExit(f"bench: {world} ranks need {world} GPUs, {ndev} visible "
                         "(FT_BENCH_SHARED_GPU=1 rehearses several ranks on one GPU)")
    return local_rank, world


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one GPU each); default: WORLD_SIZE, else 1")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sessions", type=int, default=50)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--words", type=int, default=40)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--temperature", type=float, default=0.7)
    ap.add_argument("--top-p", type=float, default=0.9)
    ap.add_argument("--no-agent", action="store_true", help="direct engine path instead of the agent")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor parallel: the N ranks form ONE engine (e.g. --model llama3-70b --tp 8); "
                         "default: data parallel, one engine per rank")
    ap.add_argument("--no-custom-allreduce", dest="custom_allreduce", action="store_false",
                    help="TP: RCCL only (default: the xGMI custom collectives for decode sizes)")
    ap.add_argument("--device", default="cuda", help="cpu runs the same path over gloo (tests)")
    ap.add_argument("--quant", default="", choices=["", "w4", "awq"],
                    help="W4A16 layer weights (the reference's AWQ-INT4 model); default bf16")
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"],
                    help="KV-cache storage (ENGINE_KV_CACHE_DTYPE): auto = bf16 (the headline), fp8 = "
                         "e4m3 at scale 1 (vLLM's --kv-cache-dtype fp8); reported in the JSON")
    ap.add_argument("--serve", choices=["door", "rank"], default="door",
                    help="DP topology: 'door' (default) = the shipping ENGINE_DP_SIZE service: every "
                         "rank is a service worker behind ONE port whose front door (rank 0, "
                         "app/server/front_door.py) places each new session on the least-loaded "
                         "worker, and every rank's load generator connects to that port; 'rank' = "
                         "each rank serves its own port to its own load generator")
    ap.add_argument("--agent-tools", type=float, default=-1.0, metavar="FRAC",
                    help="BASELINE config 5: agent with JSON-guided tool calls, FRAC of the turns "
                         "ask for a web search (stub backend); e.g. 0.2")
    a = ap.parse_args()
    if "WORLD_SIZE" not in os.environ:
        if (a.gpus or 1) > 1:
            sys.exit(_launch_ranks(a.gpus, sys.argv[1:]))
    elif a.gpus is not None and a.gpus != int(os.environ["WORLD_SIZE"]):
        raise SystemExit(f"bench: --gpus {a.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")
    if a.quant:
        os.environ["ENGINE_QUANTIZATION"] = a.quant
    if a.kv_cache_dtype != "auto":
        os.environ["ENGINE_KV_CACHE_DTYPE"] = a.kv_cache_dtype
    if a.agent_tools >= 0:
        os.environ["AGENT_GUIDED_TOOL_CALLS"] = "true"
        os.environ.setdefault("WEB_SEARCH_BACKEND", "stub")

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and os.environ.get("FT_BENCH_SHARED_GPU", "0") == "1" and \
            not os.environ.get("ENGINE_GPU_MEMORY_UTILIZATION"):
        # ranks started by torch.distributed.run (not _launch_ranks) sharing one device:
        # the same 1/n KV share each, sized against their own allocations
        os.environ["ENGINE_GPU_MEMORY_UTILIZATION"] = f"{0.85 / world:.3f}"
        os.environ.setdefault("ENGINE_KV_SIZING", "own")
    if a.tp > 1:
        return bench_tp(a, rank, world, local_rank)

    # ---- load generator child first (before this process touches the GPU) ----------
    from ws_load import client_process, summarize

    hb = {"phase": "init"}
    if rank == 0:
        _heartbeat(hb)

    port = a.port or _free_port(18100 + 10 * local_rank)
    sess_cfg = {"system_prompt": "You are a helpful voice assistant. Keep responses concise and "
                                 "conversational.",
                "temperature": a.temperature, "top_p": a.top_p, "max_tokens": a.gen,
                "ignore_eos": True}
    ctx = mp.get_context("spawn")
    parent_conn, child_conn = ctx.Pipe()
    client = ctx.Process(target=client_process, daemon=True,
                         args=(child_conn, f"ws://127.0.0.1:{port}/ws/llm", a.sessions, sess_cfg,
                               a.words, rank, a.agent_tools))
    client.start()

    # ---- service stack on this rank's GPU ------------------------------------------
    os.environ.setdefault("LOG_LEVEL", "WARNING")
    os.environ["LLM_PROVIDER"] = "native"
    os.environ["ENGINE_MODEL"] = a.model
    os.environ["ENABLE_PYDANTIC_AI"] = "false" if a.no_agent else "true"
    door = a.serve == "door"
    # door: one node-wide cap on the board (sessions may land on any worker)
    os.environ.setdefault("LLM_MAX_CONNECTIONS",
                          str(max(64, a.sessions + 8) * (world if door else 1)))
    cpu = a.device == "cpu"
    if cpu:
        os.environ["COMPUTE_DEVICE"] = "cpu"
        os.environ.setdefault("ENGINE_NUM_KV_BLOCKS", "512")
        os.environ.setdefault("ENGINE_MAX_MODEL_LEN", "2048")
    # FT_BENCH_SHARED_GPU=1: rehearse the N-rank DP path with every rank on one
    # GPU (ranks map round-robin onto the visible devices, gloo instead of RCCL,
    # which refuses two ranks on one device); the launcher sizes
    # ENGINE_GPU_MEMORY_UTILIZATION to 1/N.  The driver's multi-GPU runs leave it unset.
    shared = os.environ.get("FT_BENCH_SHARED_GPU", "0") == "1"
    dev_idx, n_dev = _device_plan(world, local_rank, a.device)
    import torch
    import torch.distributed as dist

    placement = {"rank": rank, "device": dev_idx, "pci": None, "numa_node": None, "pinned": False}
    if not cpu:
        torch.cuda.set_device(dev_idx)
        from fasttalk_llm_microservice_amd.parallel.affinity import pin_to_device

        # this rank's threads AND its load generator on the GPU's NUMA-local cores
        # (shared-GPU rehearsals leave the mask alone: the ranks would pile on one node)
        if not shared:
            placement.update(pin_to_device(dev_idx, pids=[client.pid]))
        else:
            from fasttalk_llm_microservice_amd.parallel.affinity import device_pci_address

            placement["pci"] = device_pci_address(dev_idx)
    backend = None
    if world > 1:
        backend = "gloo" if shared or cpu else "nccl"
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev_idx}"))
    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.server.asgi_aiohttp import AiohttpASGIServer
    from app.utils.config import Config

    t_init = time.time()
    cfg = Config()
    cfg.port = port
    server = WebSocketLLMServer(cfg)
    engine = server.native_handler.engine
    # capture the decode graphs the run will use before serving (a process-isolated
    # engine warms itself up before it reports ready)
    if hasattr(engine.engine, "runner") and not cpu:
        engine.engine.runner.warmup([b for b in engine.engine.runner.graph_sizes if b <= 2 * a.sessions])
    import asyncio

    asgi = AiohttpASGIServer(server.app, "127.0.0.1", port)
    loop = asyncio.new_event_loop()
    ready = threading.Event()
    board = front = None
    if door:
        # the shipping DP service (app/server/workers.py + front_door.py): rank 0 owns the
        # node board and the front door; every rank is one worker row on the board
        from app.server.front_door import DoorWorker, FrontDoor
        from app.server.node_state import NodeBoard
        from app.server.workers import _Gate

        spec = [None]
        if rank == 0:
            board = NodeBoard(world, int(os.environ["LLM_MAX_CONNECTIONS"]))
            front = FrontDoor(board, "127.0.0.1", a.port or 0).start()
            spec = [board.spec()]
        if world > 1:
            dist.broadcast_object_list(spec, src=0)
        if board is None:
            board = NodeBoard.attach(spec[0])
        board.worker_started(rank, os.getpid(), 0)
        server.connection_manager.admission = _Gate(board, rank)
        server.node, server.node_index = board, rank

    # FT_BENCH_LOOP_PROFILE=<path>: cProfile of the service event-loop thread (the asyncio
    # loop that runs the WebSocket handlers and the voice agent), dumped after the timed turns
    loop_prof_path = os.environ.get("FT_BENCH_LOOP_PROFILE")
    loop_prof = None

    def serve():
        nonlocal loop_prof
        asyncio.set_event_loop(loop)
        if loop_prof_path:
            import cProfile

            loop_prof = cProfile.Profile()
            loop_prof.enable()
        if door:
            loop.run_until_complete(asgi.start(listen=False))
            loop.run_until_complete(DoorWorker(asgi, board, rank).start())
            board.set(rank, "ready", 1)
            board.beat(rank, True)
        else:
            loop.run_until_complete(asgi.start())
        ready.set()
        loop.run_forever()

    th = threading.Thread(target=serve, daemon=True, name="asgi")
    th.start()
    if not ready.wait(120):
        raise RuntimeError("server did not start")
    if door:
        url = [None]
        if rank == 0:
            if not front.listening.wait(60):
                raise RuntimeError("front door did not open")
            url = [f"ws://127.0.0.1:{front.port}/ws/llm"]
        if world > 1:
            dist.barrier()   # every worker registered with the door
            dist.broadcast_object_list(url, src=0)
    init_s = time.time() - t_init

    def cmd(c):
        parent_conn.send(c)
        r = parent_conn.recv()
        if not r.get("ok"):
            raise RuntimeError(f"load client failed: {r.get('error')}")
        return r.get("result")

    if door:
        cmd(("url", url[0]))
    cmd("open")
    if door and world > 1:
        dist.barrier()   # every rank's sessions are placed before any turn starts
    hb["phase"] = "warmup turns"
    if a.warmup > 0:
        cmd(("run", a.warmup))
    hb["phase"] = "timed turns"

    def barrier():
        if world > 1:
            dist.barrier()
        if not cpu:
            torch.cuda.synchronize()

    barrier()
    m_before = engine.engine.metrics()
    t0 = time.perf_counter()
    res = cmd(("run", a.steps))
    barrier()
    elapsed = time.perf_counter() - t0
    hb["done"] = True
    # sessions this worker (rank) holds: the front door's placement
    placed = int(board.get(rank, "active")) if door else a.sessions
    if door and world > 1:
        # every rank reads its worker's count before any rank's load client closes its
        # sessions: the door places a rank's sessions on any worker, so a fast rank's
        # close would otherwise show up as missing sessions on a slower rank's row
        dist.barrier()
    if loop_prof is not None:
        dumped = threading.Event()

        def dump():
            loop_prof.disable()
            loop_prof.dump_stats(loop_prof_path)
            dumped.set()

        loop.call_soon_threadsafe(dump)
        dumped.wait(30)
    cmd("close")
    client.join(timeout=30)

    summ = summarize(res)
    local = {"tokens": res["tokens"], "frames": res.get("frames", 0), "elapsed": elapsed,
             "placed": placed,
             "ttft": res["ttft_s"], "tool_ttft": res.get("tool_ttft_s", []),
             "server_ttft": res.get("server_ttft_ms", []),
             "engine_ttft": res.get("engine_ttft_ms", []),
             "cached": res["cached_prompt_tokens"], "prompt": res["prompt_tokens"],
             "placement": {k: placement.get(k) for k in ("rank", "device", "pci", "numa_node", "pinned")}}
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, local)
    else:
        allr = [local]
    tokens = sum(r["tokens"] for r in allr)
    frames = sum(r["frames"] for r in allr)
    t_max = max(r["elapsed"] for r in allr)
    ttfts = sorted(x for r in allr for x in r["ttft"])
    p = lambda q: ttfts[min(len(ttfts) - 1, int(round(q * (len(ttfts) - 1))))] if ttfts else 0.0  # noqa
    value = tokens / t_max
    metrics = engine.engine.metrics()
    ctx = _timed_ctx(m_before, metrics)
    mlabel = _model_label(a.model)
    if rank == 0:
        out = {
            "metric": f"output tokens/sec (node) + p50 TTFT over WebSocket, {mlabel} at "
                      f"{a.sessions} session{'s' if a.sessions != 1 else ''}"
                      + (f" (agent, guided tool calls on {a.agent_tools:.0%} of turns)"
                         if a.agent_tools >= 0 else ""),
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": n_dev,
            "ranks": world,
            "device": a.device,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * t_max / a.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("w4a16 (bf16 compute)" if a.quant else "bf16") if not cpu else "fp32",
            "kv_cache_dtype": "fp8 (e4m3)" if a.kv_cache_dtype == "fp8" else "same as dtype",
            "data": f"synthetic (random-init {mlabel} weights, synthetic English prompts, "
                    "synthetic Llama-3 tokenizer)",
            # which GPUs the ranks ran on and over what: an N-GPU record shows by itself
            # that the collectives saw N distinct devices
            "dist_backend": ("nccl (RCCL)" if backend == "nccl" else backend) if world > 1 else None,
            "world_size": world,
            "rank_devices": [r["placement"] for r in allr],
            "distinct_gpus": len({r["placement"]["pci"] or r["placement"]["device"] for r in allr}),
            "serve": ({"mode": "front door (one port, least-loaded placement)",
                       "sessions_per_worker": [r["placed"] for r in allr]}
                      if door else {"mode": "one port per rank"}),
            "config": {"model": mlabel, "global_batch": a.sessions * world,
                       # measured context: mean tokens a decode row attended over in the
                       # timed turns (max_model_len is the engine's cap, not the workload)
                       "seq_len": ctx["ctx_mean"], "ctx_mean": ctx["ctx_mean"],
                       "ctx_max": ctx["ctx_max"], "max_model_len": engine.engine.max_model_len,
                       "parallelism": f"dp{world}",
                       "sessions_per_gpu": a.sessions, "tokens_per_turn": a.gen,
                       "path": "ws/llm -> " + ("direct engine" if a.no_agent else "voice agent") +
                               " -> in-process engine"},
            "p50_ttft_ms": round(1e3 * p(0.5), 2),
            "p99_ttft_ms": round(1e3 * p(0.99), 2),
            "p50_server_ttft_ms": _p50([x for r in allr for x in r["server_ttft"]]),
            "p50_engine_ttft_ms": _p50([x for r in allr for x in r["engine_ttft"]]),
            "per_session_tok_s": round(value / (a.sessions * world), 2),
            # WS `token` frames received vs engine tokens: < 1 means the service coalesced
            # deltas because a client fell behind (engine/sequence.py output coalescing)
            "frames": frames,
            "frames_per_token": round(frames / tokens, 4) if tokens else None,
            "reference_anchor": ("70B ~20 tok/s, ~1 s TTFT, multi-GPU (README.md:474,568)"
                                 if "70B" in mlabel else
                                 "8B single stream ~50-80 tok/s, ~200 ms TTFT on RTX 3090 (README.md:567)"),
            "prefix_cache_hit_tokens": sum(r["cached"] for r in allr),
            "prompt_tokens": sum(r["prompt"] for r in allr),
            # mean wall time between decode completions over the timed turns (engine
            # counters diffed around the timed region); *_last512 = the last 512 steps
            "engine_decode_step_ms": _timed_decode_ms(m_before, metrics),
            "engine_decode_step_ms_last512": round(metrics.get("decode_step_ms_avg", 0.0), 3),
            "engine_decode_batch_avg": round(metrics.get("decode_batch_avg", 0.0), 2),
            "kv_blocks": metrics.get("kv_blocks_total"),
            "engine_steps": {k: v for k, v in metrics.items() if k in
                             ("decode_steps", "pipelined_steps", "mixed_steps", "mixed_ahead", "pipeline_shrinks",
                              "mixed_ahead_drain")
                             or k.startswith("mixed_ahead_skip_")},
            "engine_runner": metrics.get("runner", {}),
            "engine_decode_host_ms": metrics.get("decode_host_ms", {}),
            "init_s": round(init_s, 1),
        }
        if a.agent_tools >= 0:
            # TTFT of the turns that asked for a web search (the guided call, the tool and
            # the re-prompt all sit before their first token) vs the plain turns
            tt = sorted(x for r in allr for x in r["tool_ttft"])
            pt = lambda q: tt[min(len(tt) - 1, int(round(q * (len(tt) - 1))))] if tt else 0.0  # noqa
            out["tool_turns"] = {"n": len(tt), "p50_ttft_ms": round(1e3 * pt(0.5), 2),
                                 "p99_ttft_ms": round(1e3 * pt(0.99), 2)}
            out["guided_output_tokens"] = metrics.get("guided_output_tokens", {})
            out["engine_guided"] = {k: v for k, v in metrics.items()
                                    if k in ("jump_forward_tokens", "grammar_complete_stops",
                                             "guided_pipelined_steps", "pipelined_jump_drops",
                                             "guided_capped_steps")}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    try:
        asyncio.run_coroutine_threadsafe(asgi.stop(), loop).result(timeout=15)
    except Exception:
        pass
    loop.call_soon_threadsafe(loop.stop)
    if front is not None:
        front.stop()
    if board is not None:
        board.close()
    engine.shutdown()


def _timed_ctx(before, after):
    """Mean / max context (tokens attended over) of the decode rows between two engine
    metric snapshots (engine counters; ctx_max is the run's longest, reached in the
    timed turns since histories only grow)."""
    rows = after.get("ctx_rows", 0) - before.get("ctx_rows", 0)
    toks = after.get("ctx_tokens", 0) - before.get("ctx_tokens", 0)
    return {"ctx_mean": round(toks / rows, 1) if rows > 0 else None,
            "ctx_max": after.get("ctx_max") if rows > 0 else None}


def _timed_decode_ms(before, after):
    """Mean decode step (ms) between two engine metric snapshots; None if unknown."""
    n = after.get("decode_steps", 0) - before.get("decode_steps", 0)
    t = after.get("decode_ms_sum", 0.0) - before.get("decode_ms_sum", 0.0)
    return round(t / n, 3) if n > 0 and t > 0 else None


def _model_label(name: str) -> str:
    """BASELINE.json's model names for the configs it quotes (Llama-3-8B / -70B)."""
    from fasttalk_llm_microservice_amd.models.config import resolve_model

    n = resolve_model(name).name
    return {"llama3-8b": "Llama-3-8B", "llama3.1-8b": "Llama-3.1-8B", "llama3-70b": "Llama-3-70B",
            "llama3.1-70b": "Llama-3.1-70B", "llama3.2-1b": "Llama-3.2-1B",
            "llama3.2-3b": "Llama-3.2-3B"}.get(n, n)


def bench_tp(a, rank: int, world: int, local_rank: int):
    """BASELINE config 4: one tensor-parallel engine over all ranks (RCCL/xGMI);
    rank 0 serves the WebSocket stack and drives the load, the other ranks are
    TP workers replaying rank 0's steps."""
    if a.tp != world:
        raise SystemExit(f"--tp {a.tp} needs exactly {a.tp} ranks (got {world})")
    hb = {"phase": "init"}
    if rank == 0:
        _heartbeat(hb)
    from ws_load import client_process, summarize

    port = a.port or _free_port(18100)
    sess_cfg = {"system_prompt": "You are a helpful voice assistant. Keep responses concise and "
                                 "conversational.",
                "temperature": a.temperature, "top_p": a.top_p, "max_tokens": a.gen,
                "ignore_eos": True}
    client = parent_conn = None
    if rank == 0:
        ctx = mp.get_context("spawn")
        parent_conn, child_conn = ctx.Pipe()
        client = ctx.Process(target=client_process, daemon=True,
                             args=(child_conn, f"ws://127.0.0.1:{port}/ws/llm", a.sessions, sess_cfg,
                                   a.words, 0))
        client.start()
    os.environ.setdefault("LOG_LEVEL", "WARNING")
    os.environ["LLM_PROVIDER"] = "native"
    os.environ["ENABLE_PYDANTIC_AI"] = "false" if a.no_agent else "true"
    os.environ.setdefault("LLM_MAX_CONNECTIONS", str(max(64, a.sessions + 8)))
    if a.device == "cpu":
        os.environ["COMPUTE_DEVICE"] = "cpu"
    _, n_dev = _device_plan(world, local_rank, a.device)
    import torch

    from fasttalk_llm_microservice_amd.engine.config import EngineConfig
    from fasttalk_llm_microservice_amd.engine.engine import AsyncEngine
    from fasttalk_llm_microservice_amd.parallel.tp import torchrun_tp

    t_init = time.time()
    cfg = EngineConfig.from_env(model=a.model, device=a.device, tp_size=world,
                                custom_allreduce=a.custom_allreduce,
                                tp_share_device=os.environ.get("FT_BENCH_SHARED_GPU", "0") == "1")
    if a.device == "cpu":
        cfg.num_kv_blocks = cfg.num_kv_blocks or 512
        cfg.max_model_len = min(cfg.max_model_len, 2048)
    elif cfg.tp_share_device and not cfg.num_kv_blocks:
        # every rank's weights land on one device before any rank sizes its KV pool, so
        # the free-memory rule would see the others' shards: a fixed pool per rank
        cfg.num_kv_blocks = 4096
    sync = torch.cuda.synchronize if a.device == "cuda" else (lambda: None)
    hb["phase"] = "weights + KV cache"
    eng = torchrun_tp(cfg)
    if rank != 0:
        return  # worker: returned after rank 0 sent "stop"
    hb["phase"] = "decode graph capture"
    eng.runner.warmup([b for b in eng.runner.graph_sizes if b <= 2 * a.sessions])
    aeng = AsyncEngine(eng).start()
    from app.core.websocket_server_vllm import WebSocketLLMServer
    from app.server.asgi_aiohttp import AiohttpASGIServer
    from app.utils.config import Config
    import asyncio

    scfg = Config()
    scfg.port = port
    server = WebSocketLLMServer(scfg, engine=aeng)
    asgi = AiohttpASGIServer(server.app, "127.0.0.1", port)
    loop = asyncio.new_event_loop()
    ready = threading.Event()

    # FT_BENCH_LOOP_PROFILE=<path>: cProfile of the service event-loop thread (the asyncio
    # loop that runs the WebSocket handlers and the voice agent), dumped after the timed turns
    loop_prof_path = os.environ.get("FT_BENCH_LOOP_PROFILE")
    loop_prof = None

    def serve():
        nonlocal loop_prof
        asyncio.set_event_loop(loop)
        if loop_prof_path:
            import cProfile

            loop_prof = cProfile.Profile()
            loop_prof.enable()
        loop.run_until_complete(asgi.start())
        ready.set()
        loop.run_forever()

    threading.Thread(target=serve, daemon=True, name="asgi").start()
    if not ready.wait(120):
        raise RuntimeError("server did not start")
    init_s = time.time() - t_init

    def cmd(c):
        parent_conn.send(c)
        r = parent_conn.recv()
        if not r.get("ok"):
            raise RuntimeError(f"load client failed: {r.get('error')}")
        return r.get("result")

    cmd("open")
    hb["phase"] = "warmup turns"
    if a.warmup > 0:
        cmd(("run", a.warmup))
    sync()
    hb["phase"] = "timed turns"
    m0 = eng.metrics()
    t0 = time.perf_counter()
    res = cmd(("run", a.steps))
    sync()
    elapsed = time.perf_counter() - t0
    hb["done"] = True
    if loop_prof is not None:
        dumped = threading.Event()

        def dump():
            loop_prof.disable()
            loop_prof.dump_stats(loop_prof_path)
            dumped.set()

        loop.call_soon_threadsafe(dump)
        dumped.wait(30)
    cmd("close")
    client.join(timeout=30)
    summ = summarize(res)
    metrics = eng.metrics()
    ctx = _timed_ctx(m0, metrics)
    value = res["tokens"] / elapsed
    out = {
        "metric": "output tokens/sec (node) + p50 TTFT over WebSocket, "
                  f"{a.model} TP={world} at {a.sessions} sessions",
        "value": round(value, 2), "unit": "tokens/s", "n_gpus": n_dev, "ranks": world,
        "device": a.device, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(1e3 * elapsed / a.steps, 2),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": ("w4a16 (bf16 compute)" if a.quant else "bf16") if a.device == "cuda" else "fp32",
        "kv_cache_dtype": "fp8 (e4m3)" if a.kv_cache_dtype == "fp8" else "same as dtype",
        "data": "synthetic (random-init weights, synthetic English prompts, synthetic Llama-3 tokenizer)",
        "config": {"model": a.model, "global_batch": a.sessions,
                   "seq_len": ctx["ctx_mean"], "ctx_mean": ctx["ctx_mean"], "ctx_max": ctx["ctx_max"],
                   "max_model_len": eng.max_model_len,
                   "parallelism": f"tp{world}", "custom_allreduce": a.custom_allreduce},
        "p50_ttft_ms": summ.get("p50_ttft_ms"), "p99_ttft_ms": summ.get("p99_ttft_ms"),
        "frames": res.get("frames", 0),
        "frames_per_token": round(res.get("frames", 0) / res["tokens"], 4) if res["tokens"] else None,
        "engine_decode_step_ms": round(metrics.get("decode_step_ms_avg", 0.0), 3),
        "engine_decode_batch_avg": round(metrics.get("decode_batch_avg", 0.0), 2),
        "init_s": round(init_s, 1),
    }
    print(json.dumps(out), flush=True)
    try:
        asyncio.run_coroutine_threadsafe(asgi.stop(), loop).result(timeout=15)
    except Exception:
        pass
    loop.call_soon_threadsafe(loop.stop)
    aeng.shutdown()


if __name__ == "__main__":
    main()
