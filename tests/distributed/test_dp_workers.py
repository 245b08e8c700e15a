"""DP serving as N service worker processes on one port (app/server/workers.py,
ENGINE_DP_MODE=workers): the parent's front door (app/server/front_door.py) places
every session on the least-loaded worker, each streams from its own engine, and a
killed worker is restarted and serves again.  CPU only: the engines use the
synthetic runner (ENGINE_SYNTHETIC_STEP_MS)."""
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
        # the front door balanced the sessions: 8 + 8, every run
        assert r["probe"] == [8, 8], r["probe"]
        assert pool.door is not None and pool.door.stats["per_worker"][0] >= 8
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


def _http_json(port, path):
    import json
    import urllib.error
    import urllib.request

    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{port}{path}", timeout=10) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def _wait_health(port, code, timeout=120):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            st, body = _http_json(port, "/health")
            if st == code:
                return body
        except OSError:
            pass
        time.sleep(0.3)
    raise TimeoutError(f"/health never answered {code}")


def test_dp_workers_behave_as_one_service(monkeypatch):
    """(i) the node-wide LLM_MAX_CONNECTIONS cap, (ii) the parent's
    :9092 /metrics counts generations from every worker, /stats sums them, (iii) a
    killed worker turns /health 503 on the survivors until it is back."""
    import json

    import aiohttp

    from app.monitoring.service_monitor import MonitoringServer, ServiceMonitor
    from app.server.workers import WorkerPool

    for k, v in {"ENGINE_SYNTHETIC_STEP_MS": "2", "COMPUTE_DEVICE": "cpu", "LLM_PROVIDER": "native",
                 "ENGINE_MODEL": "tiny", "ENABLE_PYDANTIC_AI": "false", "LOG_LEVEL": "WARNING",
                 "LLM_MAX_CONNECTIONS": "5"}.items():
        monkeypatch.setenv(k, v)
    port = _free_port()
    pool = WorkerPool(2, "127.0.0.1", port, max_restarts=1, max_connections=5)
    mon = ServiceMonitor()
    mon.attach_node(pool.board)
    ms = MonitoringServer(port=0, monitor=mon).app.test_client()
    pool.start()
    try:
        assert pool.wait_ready(180)
        body = _wait_health(port, 200)
        assert len(body["workers"]) == 2 and all(w["ready"] for w in body["workers"])

        # (i) 5 sessions fill the node whichever worker accepted them; the 6th is refused
        async def cap():
            async with aiohttp.ClientSession() as s:
                socks = []
                for _ in range(5):
                    ws = await s.ws_connect(f"ws://127.0.0.1:{port}/ws/llm")
                    assert json.loads((await ws.receive()).data)["type"] == "session_started"
                    socks.append(ws)
                extra = await s.ws_connect(f"ws://127.0.0.1:{port}/ws/llm")
                refused = json.loads((await extra.receive()).data)
                await extra.close()
                st, stats = _http_json(port, "/stats")
                await socks[0].close()
                await asyncio.sleep(0.5)
                again = await s.ws_connect(f"ws://127.0.0.1:{port}/ws/llm")
                ok = json.loads((await again.receive()).data)
                for ws in socks[1:] + [again]:
                    await ws.close()
                return refused, stats, ok
        refused, stats, ok = asyncio.run(cap())
        assert refused["type"] == "error" and refused["error"]["code"] == "max_connections"
        assert stats["connections"]["active_connections"] == 5
        assert stats["connections"]["max_connections"] == 5
        assert ok["type"] == "session_started", "a closed session must free its slot"

        # (ii) generations from both workers reach the parent's monitor and /stats
        time.sleep(1.0)
        r = _sessions(port, 4, turns=2)
        assert r["turns"] == 8
        time.sleep(1.5)   # two snapshot periods
        m = ms.get("/metrics").get_json()
        assert m["generations"] == 8 and m["total_tokens_generated"] == 8 * 6, m
        per = [w["generations"] for w in m["workers"]]
        # 4 sessions x 2 turns placed by the front door: 2 sessions per worker
        assert per == [4, 4], per
        st, stats = _http_json(port, "/stats")
        assert stats["connections"]["total_generations_completed"] == 8
        assert b"fasttalk_worker_ready" in ms.get("/metrics/prometheus").data

        # (iii) a dead worker: 503 on the survivor until the respawned worker serves
        victim = pool.procs[0]
        victim.kill()
        victim.join(10)
        pool.supervise_once()
        body = _wait_health(port, 503, timeout=30)
        assert not body["workers"][0]["ready"] and body["status"] == "degraded"
        body = _wait_health(port, 200, timeout=180)
        assert body["workers"][0]["restarts"] == 1
        r = _sessions(port, 4)
        assert r["turns"] == 4
    finally:
        pool.stop()
        pool.close()


def test_dp_worker_startup_check_fails_before_serving(monkeypatch):
    """A worker whose backend is unreachable exits 1 before opening the port
    (reference websocket_launcher.py:104-105); the pool reports the failed start."""
    from app.server.workers import STARTUP_FAILED, WorkerPool

    dead = _free_port()
    for k, v in {"LLM_PROVIDER": "vllm", "VLLM_BASE_URL": f"http://127.0.0.1:{dead}/v1",
                 "ENABLE_PYDANTIC_AI": "false", "LOG_LEVEL": "WARNING", "COMPUTE_DEVICE": "cpu"}.items():
        monkeypatch.setenv(k, v)
    port = _free_port()
    pool = WorkerPool(1, "127.0.0.1", port, max_restarts=0).start()
    try:
        assert not pool.wait_ready(120)
        pool.procs[0].join(10)
        assert pool.procs[0].exitcode == STARTUP_FAILED
        with pytest.raises(OSError):
            socket.create_connection(("127.0.0.1", port), timeout=1).close()
    finally:
        pool.stop()
        pool.close()


def test_dp_tp_workers_own_disjoint_gpu_ranges():
    """DP x TP: worker i's TP group starts at GPU i*tp (ENGINE_DEVICE_BASE, read by
    AsyncEngine.from_config) and its ranks take the next tp GPUs; the workers of an
    8-GPU node partition it."""
    from app.server.workers import worker_env
    from fasttalk_llm_microservice_amd.parallel.tp import tp_device_index

    for dp, tp in ((8, 1), (4, 2), (2, 4), (1, 8)):
        owned = []
        for i in range(dp):
            env = worker_env(i, dp, tp)
            assert env["ENGINE_DP_SIZE"] == "1"
            base = int(env["ENGINE_DEVICE_BASE"])
            assert base == i * tp
            devs = [tp_device_index(base, r) for r in range(tp)]
            assert devs == list(range(i * tp, (i + 1) * tp))
            owned += devs
        assert sorted(owned) == list(range(8))
    # ranks that share one device (rehearsals) all sit on the base
    assert {tp_device_index(4, r, share_device=True) for r in range(4)} == {4}


def test_front_door_balances_refuses_and_reroutes(tmp_path):
    """The door alone, with fake workers on its control socket: least-loaded placement
    (pending hand-offs count before a worker reports), 503 with no worker ready, and a
    worker whose control socket died is routed around."""
    import json
    import socket as _s
    import urllib.request

    from app.server.front_door import FrontDoor
    from app.server.node_state import NodeBoard

    board = NodeBoard(3, 100)
    door = FrontDoor(board, "127.0.0.1", 0).start()
    ctl = []
    try:
        for i in range(3):
            c = _s.socket(_s.AF_UNIX, _s.SOCK_SEQPACKET)
            c.connect(door.ctl_path)
            c.sendall(f"W{i}\n".encode())
            ctl.append(c)
            board.worker_started(i, 1000 + i, 0)
        assert door.listening.wait(10)
        port = door.port
        # not ready yet: the door answers 503
        with pytest.raises(urllib.error.HTTPError) as e:
            urllib.request.urlopen(f"http://127.0.0.1:{port}/health", timeout=5)
        assert e.value.code == 503 and json.loads(e.value.read())["status"] == "unavailable"
        for i in range(3):
            board.set(i, "ready", 1)
            board.beat(i, True)
        board.set(0, "conns", 5)          # worker 0 already busy
        clients = [_s.create_connection(("127.0.0.1", port)) for _ in range(6)]
        got = [[] for _ in range(3)]
        deadline = time.time() + 10
        while sum(map(len, got)) < 6 and time.time() < deadline:
            for i, c in enumerate(ctl):
                c.settimeout(0.05)
                try:
                    msg, fds, _, _ = _s.recv_fds(c, 16, 4)
                except (TimeoutError, _s.timeout, BlockingIOError):
                    continue
                got[i] += fds
        counts = [len(g) for g in got]
        # nothing reported back yet: the six hand-offs split 0 / 3 / 3 (worker 0 had 5)
        assert counts == [0, 3, 3], counts
        for g in got:
            for fd in g:
                os.close(fd)
        # worker 1 (the least loaded) loses its control socket: the door tries it, fails
        # and routes the connection to worker 2 instead
        board.set(2, "conns", 1)
        ctl[1].close()
        extra = _s.create_connection(("127.0.0.1", port))
        time.sleep(0.5)
        ctl[2].settimeout(2)
        msg, fds, _, _ = _s.recv_fds(ctl[2], 16, 4)
        assert len(fds) == 1 and door.stats["rerouted"] >= 1
        os.close(fds[0])
        # a worker alive and ready but whose heartbeat went stale (event loop stalled)
        # gets no new sessions: worker 0 is idle now, yet the next one goes to worker 2
        board.set(0, "conns", 0)
        board.set(0, "heartbeat", time.time() - 60)
        late = _s.create_connection(("127.0.0.1", port))
        time.sleep(0.5)
        msg, fds, _, _ = _s.recv_fds(ctl[2], 16, 4)
        assert len(fds) == 1
        os.close(fds[0])
        ctl[0].settimeout(0.2)
        with pytest.raises((TimeoutError, _s.timeout, BlockingIOError)):
            _s.recv_fds(ctl[0], 16, 4)
        for c in clients + [extra, late]:
            c.close()
    finally:
        door.stop()
        for c in ctl:
            c.close()
        board.close()
