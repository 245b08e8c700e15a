"""WebSocket load generator for ``/ws/llm`` (aiohttp client; the ``websockets``
package is not installed).

Each simulated user keeps ONE WebSocket session for the whole run (conversation
history accumulates turn after turn, like a voice session) and, per turn, sends
a ``user_message`` then reads ``token`` frames until ``response_complete``.
Measured per turn: time to first token frame (client clock), output tokens
(engine count from ``response_complete.stats.tokens_generated``), frames.

Used in-process by ``bench.py`` (``LoadClient`` in a child process driven over a
pipe) and standalone against a running server:

    python bench/ws_load.py --url ws://127.0.0.1:8000/ws/llm --sessions 50 --turns 4
"""
from __future__ import annotations

import argparse
import asyncio
import json
import random
import statistics
import time
from typing import Any, Dict, List, Optional

WORDS = ("the voice assistant should answer quickly and naturally about weather news travel music "
         "sports cooking history science movies books health fitness coffee tea morning evening "
         "weekend plans family friends city river mountain ocean garden computer phone battery "
         "meeting schedule reminder question answer story idea project update please thanks").split()


# words that never trigger the agent's tool heuristics (app/agents/voice_agent.py _TOOL_HINTS)
PLAIN_WORDS = tuple(w for w in WORDS if w not in ("news", "weather", "question", "answer",
                                                  "schedule", "reminder", "update"))


def user_text(rng: random.Random, words: int, tool_frac: float = -1.0) -> str:
    """A synthetic user turn.  ``tool_frac >= 0`` (agent tool-calling bench, BASELINE
    config 5): that fraction of turns asks for a web search, the rest are plain
    chat with no tool-hint words."""
    if tool_frac < 0:
        return " ".join(rng.choice(WORDS) for _ in range(words)).capitalize() + "?"
    if rng.random() < tool_frac:
        topic = " ".join(rng.choice(PLAIN_WORDS) for _ in range(max(1, words // 4)))
        return f"Search the web for the latest news about {topic}?"
    return " ".join(rng.choice(PLAIN_WORDS) for _ in range(words)).capitalize() + "."


class Session:
    def __init__(self, idx: int, url: str, cfg: Dict[str, Any], words: int, seed: int,
                 tool_frac: float = -1.0):
        self.idx = idx
        self.tool_frac = tool_frac
        self.url = url
        self.cfg = cfg
        self.words = words
        self.rng = random.Random(seed * 7919 + idx)
        self.ws = None
        self.http = None
        self.turns: List[Dict[str, Any]] = []

    async def open(self, http):
        self.http = http
        self.ws = await http.ws_connect(self.url, max_msg_size=0, heartbeat=None)
        m = await self.ws.receive_json()
        assert m["type"] == "session_started", m
        await self.ws.send_json({"type": "start_session", "config": self.cfg})
        m = await self.ws.receive_json()
        assert m["type"] == "session_configured", m

    async def turn(self) -> Dict[str, Any]:
        t0 = time.perf_counter()
        text = user_text(self.rng, self.words, self.tool_frac)
        await self.ws.send_json({"type": "user_message", "text": text})
        first = None
        frames = 0
        while True:
            msg = await self.ws.receive()
            m = json.loads(msg.data)
            t = m.get("type")
            if t == "token":
                frames += 1
                if first is None:
                    first = time.perf_counter() - t0
            elif t == "response_complete":
                st = m["stats"]
                rec = {"ttft_s": first if first is not None else time.perf_counter() - t0,
                       "latency_s": time.perf_counter() - t0, "frames": frames,
                       "tokens": int(st.get("tokens_generated", frames)),
                       "server_ttft_ms": st.get("ttft_ms"),
                       "engine_ttft_ms": st.get("engine_ttft_ms"),
                       "cached_prompt_tokens": st.get("cached_prompt_tokens", 0),
                       "prompt_tokens": st.get("prompt_tokens", 0),
                       # a turn that asks for a web search (config 5: the agent's tool round)
                       "tool": text.startswith("Search the web")}
                self.turns.append(rec)
                return rec
            elif t == "error":
                raise RuntimeError(f"session {self.idx}: server error {m}")

    async def close(self):
        if self.ws is not None:
            try:
                await self.ws.send_json({"type": "end_session"})
                await asyncio.wait_for(self.ws.receive(), 5)
            except Exception:
                pass
            await self.ws.close()


class LoadClient:
    def __init__(self, url: str, sessions: int, cfg: Dict[str, Any], words: int = 40, seed: int = 0,
                 tool_frac: float = -1.0):
        self.tool_frac = tool_frac
        self.url = url
        self.n = sessions
        self.cfg = cfg
        self.words = words
        self.seed = seed
        self.sessions: List[Session] = []
        self.http = None

    async def open(self):
        import aiohttp

        self.http = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None),
                                          connector=aiohttp.TCPConnector(limit=0))  # WS: no pool cap
        self.sessions = [Session(i, self.url, self.cfg, self.words, self.seed, self.tool_frac)
                         for i in range(self.n)]
        await asyncio.gather(*[s.open(self.http) for s in self.sessions])

    async def run_turns(self, turns: int) -> Dict[str, Any]:
        t0 = time.perf_counter()

        async def one(s: Session):
            out = []
            for _ in range(turns):
                out.append(await s.turn())
            return out

        res = await asyncio.gather(*[one(s) for s in self.sessions])
        dt = time.perf_counter() - t0
        recs = [r for rs in res for r in rs]
        return {"elapsed_s": dt, "tokens": sum(r["tokens"] for r in recs),
                "frames": sum(r["frames"] for r in recs), "ttft_s": [r["ttft_s"] for r in recs],
                "tool_ttft_s": [r["ttft_s"] for r in recs if r["tool"]],
                "latency_s": [r["latency_s"] for r in recs],
                "server_ttft_ms": [r["server_ttft_ms"] for r in recs if r["server_ttft_ms"] is not None],
                "engine_ttft_ms": [r["engine_ttft_ms"] for r in recs if r["engine_ttft_ms"] is not None],
                "cached_prompt_tokens": sum(r["cached_prompt_tokens"] or 0 for r in recs),
                "prompt_tokens": sum(r["prompt_tokens"] or 0 for r in recs), "turns": len(recs)}

    async def close(self):
        await asyncio.gather(*[s.close() for s in self.sessions], return_exceptions=True)
        if self.http is not None:
            await self.http.close()


def client_process(conn, url: str, sessions: int, cfg: Dict[str, Any], words: int, seed: int,
                   tool_frac: float = -1.0):
    """Child-process entry: commands over a pipe ('open', ('run', n), 'close')."""
    loop = asyncio.new_event_loop()
    asyncio.set_event_loop(loop)
    lc = LoadClient(url, sessions, cfg, words, seed, tool_frac)
    try:
        while True:
            cmd = conn.recv()
            try:
                if cmd == "open":
                    loop.run_until_complete(lc.open())
                    conn.send({"ok": True})
                elif isinstance(cmd, tuple) and cmd[0] == "url":   # before "open"
                    lc.url = cmd[1]
                    conn.send({"ok": True})
                elif isinstance(cmd, tuple) and cmd[0] == "run":
                    conn.send({"ok": True, "result": loop.run_until_complete(lc.run_turns(cmd[1]))})
                elif cmd == "close":
                    loop.run_until_complete(lc.close())
                    conn.send({"ok": True})
                    return
            except Exception as e:  # report, keep serving
                conn.send({"ok": False, "error": repr(e)})
    finally:
        loop.close()


def summarize(r: Dict[str, Any]) -> Dict[str, Any]:
    t = sorted(r["ttft_s"])
    pct = lambda q: t[min(len(t) - 1, int(round(q * (len(t) - 1))))] if t else 0.0  # noqa: E731
    return {"tokens_per_s": r["tokens"] / r["elapsed_s"], "tokens": r["tokens"],
            "elapsed_s": r["elapsed_s"], "turns": r["turns"], "p50_ttft_ms": 1e3 * pct(0.5),
            "p99_ttft_ms": 1e3 * pct(0.99),
            "mean_latency_s": statistics.fmean(r["latency_s"]) if r["latency_s"] else 0.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="ws://127.0.0.1:8000/ws/llm")
    ap.add_argument("--sessions", type=int, default=50)
    ap.add_argument("--turns", type=int, default=3)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--words", type=int, default=40)
    ap.add_argument("--temperature", type=float, default=0.7)
    a = ap.parse_args()
    cfg = {"system_prompt": "You are a helpful voice assistant. Keep responses concise and conversational.",
           "temperature": a.temperature, "top_p": 0.9, "max_tokens": a.max_tokens, "ignore_eos": True}

    async def go():
        lc = LoadClient(a.url, a.sessions, cfg, a.words)
        await lc.open()
        r = await lc.run_turns(a.turns)
        await lc.close()
        return r

    print(json.dumps(summarize(asyncio.run(go())), indent=1))


if __name__ == "__main__":
    main()
