"""Data-parallel serving inside one service (SURVEY.md §2.6 P2 "DP replicas +
session-affinity router"): ``ENGINE_DP_SIZE=N`` runs N engine replicas, each in
its own process on its own GPU(s) (replica i owns GPUs [i*tp, (i+1)*tp), and
``ENGINE_TP_SIZE>1`` makes each replica a TP group of its own).

The router keeps every conversation on the replica that already holds its KV
blocks (multi-turn prefix reuse only works there) and sends a new conversation
to the replica with the fewest active requests.  It exposes the AsyncEngine
surface (``generate`` / ``abort`` / ``is_healthy`` / ``model_info`` and an
``engine`` facade with tokenizer, chat template and aggregated ``metrics()``)
so :class:`app.core.native_handler.NativeHandler` cannot tell the difference.

Replica protocol (``multiprocessing`` pipe, both directions pickled):
  router -> replica: ("add", rid, prompt_ids, params) | ("abort", rid) | ("stop",)
  replica -> router: ("ready", info) | ("out", [RequestOutput...], metrics) | ("dead", err)

Failure handling (SURVEY.md §5 "TP worker death -> health 503 + engine
restart"): a replica whose engine cannot step again -- a TP worker process died,
the step loop stalled, a fatal device error -- reports ``dead`` and exits (its
TP workers follow their parent).  The router fails that replica's requests, is
unhealthy (``/health`` 503) while it respawns the replica in a fresh process
(``max_restarts`` times), and routes new conversations to live replicas.
"""
from __future__ import annotations

import asyncio
import collections
import itertools
import logging
import multiprocessing as mp
import os
import threading
import time
import uuid
from typing import Any, AsyncIterator, Dict, List, Optional, Sequence as Seq

from ..engine.chat_template import ChatTemplate
from ..engine.engine import EngineError
from ..engine.sequence import RequestOutput, coalesce
from ..engine.tokenizer import get_tokenizer
from ..models.config import resolve_model

log = logging.getLogger("fasttalk.dp")


def _replica_watchdog(eng, send, beat, stall_s: float):
    """Replica-side liveness: exits the process (after reporting ``dead``) when a
    TP worker died, the step loop has been stuck for ``stall_s`` while busy, or
    the router process is gone.  A step stuck inside a collective cannot notice
    any of these itself."""
    ppid = os.getppid()

    def watch():
        while True:
            time.sleep(0.5)
            why = None
            group = getattr(eng, "tp_group", None)
            if group is not None and hasattr(group, "alive") and not group.alive():
                why = "a tensor-parallel worker process died"
            elif beat[1] and time.time() - beat[0] > stall_s:
                why = f"engine step stalled for more than {stall_s:.0f}s"
            elif os.getppid() != ppid:
                os._exit(3)
            if why:
                log.error("replica: %s; exiting for a restart", why)
                try:
                    send(("dead", why))
                finally:
                    os._exit(3)

    threading.Thread(target=watch, name="fasttalk-replica-watch", daemon=True).start()


def _replica_main(index: int, cfg, conn, device_base: int = 0):
    """Replica process: one engine (TP group when cfg.tp_size > 1) + step loop."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from ..engine.engine import AsyncEngine

    try:
        base = device_base + index * max(1, cfg.tp_size)
        if cfg.resolved_device() == "cuda":
            import torch

            torch.cuda.set_device(base)
            from .affinity import pin_to_device

            pin_to_device(base)
        if cfg.tp_size > 1:
            from .tp import spawn_tp_engine

            eng = spawn_tp_engine(cfg, device_base=base)
        else:
            from ..engine.engine import LLMEngine

            eng = LLMEngine(cfg)
        if cfg.resolved_device() == "cuda" and not cfg.enforce_eager and hasattr(eng.runner, "warmup"):
            eng.runner.warmup()
    except BaseException as e:  # pragma: no cover - reported to the router
        conn.send(("dead", repr(e)))
        return
    lock = threading.Lock()

    def send(msg):
        with lock:
            conn.send(msg)

    send(("ready", {"num_blocks": eng.bm.num_blocks, "max_model_len": eng.max_model_len}))
    beat = [time.time(), False]  # last loop iteration, busy
    _replica_watchdog(eng, send, beat, float(os.environ.get("ENGINE_STALL_S", "120")))
    outs: List[RequestOutput] = []
    last_metrics = 0.0
    streak = 0
    try:
        while True:
            beat[0], beat[1] = time.time(), eng.has_work()
            timeout = 0.0 if eng.has_work() else 0.05
            while conn.poll(timeout):
                cmd = conn.recv()
                timeout = 0.0
                if cmd[0] == "add":
                    _, rid, prompt, params = cmd
                    try:
                        eng.add_request(rid, prompt, params, on_output=outs.append)
                    except Exception as e:
                        outs.append(RequestOutput(rid, "", [], finished=True, finish_reason="error",
                                                  error=str(e)))
                elif cmd[0] == "warm":  # background prefix warm-up: optional work
                    _, rid, prompt = cmd
                    try:
                        from ..engine.sampling_params import SamplingParams

                        eng.add_request(rid, prompt, SamplingParams(temperature=0.0, max_tokens=1),
                                        background=True)
                    except Exception as e:
                        log.warning("prefix warm-up %s not queued: %s", rid, e)
                elif cmd[0] == "abort":
                    eng.abort(cmd[1])
                elif cmd[0] == "stop":
                    return
            if eng.has_work():
                try:
                    eng.step()
                    streak = 0
                except Exception as e:  # same contract as AsyncEngine._run
                    log.exception("replica step failed")
                    from ..engine.runner import CommFault

                    # error outputs land in `outs`; a collective fault may have left
                    # KV from partial sums in committed blocks: drop the prefix cache
                    eng.fail_unfinished(str(e), reset_cache=isinstance(e, CommFault))
                    streak += 1
                    if not AsyncEngine._recoverable(e) or streak >= int(
                            os.environ.get("ENGINE_MAX_FAIL_STREAK", "3")):
                        if outs:
                            send(("out", list(outs), None))
                        send(("dead", repr(e)))
                        return
            now = time.time()
            metrics = None
            if now - last_metrics > 0.5:
                metrics = eng.metrics()
                last_metrics = now
            if outs or metrics is not None:
                send(("out", list(outs), metrics))
                outs.clear()  # the sequences' on_output callbacks append to this list
    finally:
        eng.shutdown()


class _Replica:
    def __init__(self, index: int, cfg, ctx, device_base: int = 0):
        self.index = index
        self.conn, child = ctx.Pipe()
        # not a daemon: a TP replica spawns its worker processes.  The replica exits
        # by itself when the router process is gone (_replica_watchdog) and the
        # router stops it at interpreter exit (MultiGPUEngine.start registers that)
        self.proc = ctx.Process(target=_replica_main, args=(index, cfg, child, device_base),
                                daemon=False, name=f"fasttalk-dp{index}")
        self.proc.start()
        child.close()
        self.lock = threading.Lock()
        self.active = 0
        self.metrics: Dict[str, Any] = {}
        self.info: Dict[str, Any] = {}
        self.error: Optional[str] = None

    def send(self, msg):
        with self.lock:
            self.conn.send(msg)


class _Facade:
    """What NativeHandler / the server read from ``engine.engine``."""

    def __init__(self, router: "MultiGPUEngine", cfg):
        self._router = router
        self.cfg = cfg
        self.model_cfg = resolve_model(cfg.weights if cfg.weights not in ("random", None, "")
                                       else cfg.model)
        tok_path = cfg.tokenizer or (cfg.weights if cfg.weights not in ("random", None, "") else None)
        self.tokenizer = get_tokenizer(tok_path)
        self.template = ChatTemplate(self.tokenizer)
        self.max_model_len = min(cfg.max_model_len, self.model_cfg.max_position_embeddings)

    def token_trie(self):
        from ..runtime import rt

        if getattr(self, "_trie", None) is None:
            self._trie = rt().TokenTrie(self.tokenizer.id_to_bytes)
        return self._trie

    def metrics(self) -> Dict[str, Any]:
        reps = [r.metrics for r in self._router.replicas]
        agg: Dict[str, Any] = dict(reps[0]) if len(reps) == 1 else {}
        agg.update({"replicas": len(reps), "per_replica": reps})
        for key in ("running", "waiting", "kv_blocks_total", "kv_blocks_free", "generated_tokens",
                    "prefill_tokens", "requests", "preemptions"):
            agg[key] = sum(int(m.get(key, 0) or 0) for m in reps)
        tot = agg["kv_blocks_total"]
        agg["kv_usage"] = 1.0 - agg["kv_blocks_free"] / tot if tot else 0.0
        return agg


class MultiGPUEngine:
    """``dp_size`` engine replicas in child processes.  With ``dp_size == 1`` it is
    the process-isolated single engine (``ENGINE_SEPARATE_PROCESS``): the step loop
    no longer shares a GIL with the WebSocket event loop."""

    def __init__(self, cfg, device_base: Optional[int] = None):
        self.cfg = cfg
        if device_base is None and os.environ.get("ENGINE_DEVICE_BASE"):
            device_base = int(os.environ["ENGINE_DEVICE_BASE"])   # a DP service worker's GPUs
        if device_base is None:
            device_base = int(os.environ.get("LOCAL_RANK", "0")) * max(1, cfg.dp_size) * \
                max(1, cfg.tp_size) if cfg.resolved_device() == "cuda" else 0
        self.device_base = device_base
        self.dp = max(1, cfg.dp_size)
        self.ctx = mp.get_context("spawn")
        self.replicas: List[_Replica] = []
        self.engine = _Facade(self, cfg)
        self._streams: Dict[str, asyncio.Queue] = {}
        self._loops: Dict[str, asyncio.AbstractEventLoop] = {}
        self._owner: Dict[str, _Replica] = {}
        self._affinity: "collections.OrderedDict[str, int]" = collections.OrderedDict()
        self._ids = itertools.count()
        self._readers: List[threading.Thread] = []
        self._stop = False
        self.restarts = 0

    # ------------------------------------------------------------------ lifecycle
    @staticmethod
    def _await_ready(r: _Replica, timeout: float):
        t0 = time.time()
        while not r.conn.poll(1.0):
            if not r.proc.is_alive() or time.time() - t0 > timeout:
                raise EngineError(f"DP replica {r.index} failed to start")
        kind, payload = r.conn.recv()
        if kind != "ready":
            raise EngineError(f"DP replica {r.index} failed: {payload}")
        r.info = payload

    def _start_reader(self, r: _Replica):
        th = threading.Thread(target=self._reader, args=(r,), daemon=True,
                              name=f"fasttalk-dp-reader{r.index}")
        th.start()
        self._readers.append(th)

    def start(self, timeout: float = 1800.0):
        import atexit

        atexit.register(self.shutdown)
        self.replicas = [_Replica(i, self.cfg, self.ctx, self.device_base) for i in range(self.dp)]
        t0 = time.time()
        for r in self.replicas:
            self._await_ready(r, timeout)
        for r in self.replicas:
            self._start_reader(r)
        log.info("DP engine: %d replicas ready in %.1fs", self.dp, time.time() - t0)
        return self

    def _replica_down(self, r: _Replica):
        """Fails the replica's requests and respawns it in a fresh process (the old
        one, and with it its TP workers, exits); unhealthy until the new one is ready."""
        self._fail_replica(r)
        if self._stop or self.restarts >= max(0, int(getattr(self.cfg, "max_restarts", 0))):
            return
        self.restarts += 1
        threading.Thread(target=self._restart, args=(r,), daemon=True,
                         name=f"fasttalk-dp-restart{r.index}").start()

    def _restart(self, old: _Replica, timeout: float = 1800.0):
        old.proc.join(timeout=10)
        if old.proc.is_alive():
            old.proc.kill()
            old.proc.join(timeout=10)
        time.sleep(float(os.environ.get("ENGINE_RESTART_DELAY", "2")))  # workers' exit frees the GPU
        if self._stop:
            return
        log.warning("restarting DP replica %d (restart %d/%d) after: %s", old.index, self.restarts,
                    self.cfg.max_restarts, old.error)
        new = _Replica(old.index, self.cfg, self.ctx, self.device_base)
        try:
            self._await_ready(new, timeout)
        except Exception as e:
            new.error = str(e)
            self.replicas[old.index] = new
            log.error("DP replica %d did not come back: %s", old.index, e)
            return
        self.replicas[old.index] = new
        self._start_reader(new)
        log.warning("DP replica %d is back", old.index)

    def shutdown(self):
        if self._stop:
            return
        self._stop = True
        for r in self.replicas:
            try:
                r.send(("stop",))
            except Exception:
                pass
        for r in self.replicas:
            r.proc.join(timeout=30)
            if r.proc.is_alive():
                r.proc.terminate()

    def is_healthy(self, stall_s: float = 120.0) -> bool:
        return bool(self.replicas) and all(r.proc.is_alive() and r.error is None
                                           for r in self.replicas)

    # ------------------------------------------------------------------ plumbing
    def _reader(self, r: _Replica):
        while not self._stop:
            try:
                msg = r.conn.recv()
            except (EOFError, OSError):
                r.error = r.error or "replica exited"
                self._replica_down(r)
                return
            if msg[0] == "out":
                _, outs, metrics = msg
                if metrics is not None:
                    r.metrics = metrics
                by_loop: Dict[asyncio.AbstractEventLoop, list] = {}
                for o in outs:
                    loop = self._loops.get(o.request_id)
                    if loop is not None:
                        by_loop.setdefault(loop, []).append(o)
                for loop, items in by_loop.items():
                    try:
                        loop.call_soon_threadsafe(self._dispatch, items)
                    except RuntimeError:
                        pass
            elif msg[0] == "dead":
                r.error = msg[1]
                self._replica_down(r)
                return

    def _fail_replica(self, r: _Replica):
        for rid, owner in list(self._owner.items()):
            if owner is r:
                loop = self._loops.get(rid)
                if loop is not None:
                    err = RequestOutput(rid, "", [], finished=True, finish_reason="error",
                                        error=f"DP replica {r.index} failed: {r.error}")
                    try:
                        loop.call_soon_threadsafe(self._dispatch, [err])
                    except RuntimeError:
                        pass

    def _dispatch(self, items: List[RequestOutput]):
        for o in items:
            q = self._streams.get(o.request_id)
            if q is not None:
                q.put_nowait(o)

    def _pick(self, rid: str) -> _Replica:
        key = rid.split("#", 1)[0]
        idx = self._affinity.get(key)
        if idx is None or self.replicas[idx].error is not None:
            live = [r for r in self.replicas if r.error is None] or self.replicas
            idx = min(live, key=lambda r: r.active).index
            self._affinity[key] = idx
            while len(self._affinity) > 100_000:
                self._affinity.popitem(last=False)
        else:
            self._affinity.move_to_end(key)
        return self.replicas[idx]

    # ------------------------------------------------------------------ public API
    def new_request_id(self) -> str:
        return f"dp-{next(self._ids)}-{uuid.uuid4().hex[:6]}"

    async def generate(self, prompt_ids: Seq[int], params, request_id: Optional[str] = None
                       ) -> AsyncIterator[RequestOutput]:
        rid = request_id or self.new_request_id()
        if rid in self._streams:
            raise EngineError(f"duplicate request id {rid}")
        rep = self._pick(rid)
        if rep.error is not None:
            raise EngineError(f"DP replica {rep.index} failed: {rep.error}")
        q: asyncio.Queue = asyncio.Queue()
        self._streams[rid] = q
        self._loops[rid] = asyncio.get_running_loop()
        self._owner[rid] = rep
        rep.active += 1
        finished = False
        try:
            rep.send(("add", rid, list(prompt_ids), params))
            while True:
                o = coalesce(await q.get(), q)
                finished = o.finished
                yield o
                if finished:
                    break
        finally:
            rep.active -= 1
            self._streams.pop(rid, None)
            self._loops.pop(rid, None)
            self._owner.pop(rid, None)
            if not finished and rep.error is None:
                try:
                    rep.send(("abort", rid))
                except Exception:
                    pass

    def prefill_background(self, prompt_ids: Seq[int], session_id: Optional[str] = None) -> str:
        """AsyncEngine.prefill_background across replicas: the warm-up goes to the
        replica the session's turns are affine to (its prefix cache is the one the
        next turn will hit).  Fire and forget: a warm-up produces no output."""
        rid = f"{session_id}#warm-{next(self._ids)}" if session_id else self.new_request_id()
        rep = self._pick(rid)
        if rep.error is None:
            try:
                rep.send(("warm", rid, list(prompt_ids)))
            except Exception:  # optional work: never fails a session
                pass
        return rid

    def abort(self, request_id: str) -> bool:
        rep = self._owner.get(request_id)
        if rep is None:
            return False
        rep.send(("abort", request_id))
        return True

    def active_requests(self) -> List[str]:
        return list(self._owner)

    def model_info(self) -> Dict[str, Any]:
        m = self.engine.model_cfg
        return {
            "model": m.name, "num_layers": m.num_layers, "hidden_size": m.hidden_size,
            "num_heads": m.num_heads, "num_kv_heads": m.num_kv_heads, "vocab_size": m.vocab_size,
            "max_model_len": self.engine.max_model_len, "weights": self.cfg.weights,
            "tensor_parallel_size": self.cfg.tp_size, "data_parallel_size": self.dp,
            "kv_cache_tokens": sum(r.info.get("num_blocks", 0) for r in self.replicas) *
            self.cfg.block_size,
        }
