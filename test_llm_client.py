#!/usr/bin/env python3
"""Manual /ws/llm client (the reference ships an interactive one,
``test_llm_client.py:13-155``).  It checks ``/health``, opens a session,
streams replies token by token and prints the per-turn stats.  aiohttp is used
because the ``websockets`` package is not part of this stack.

    python test_llm_client.py                       # interactive prompt loop
    python test_llm_client.py -m "Hi" -m "And?"     # scripted turns, then exit
    python test_llm_client.py --url ws://host:8000/ws/llm --max-tokens 64
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
import time

import aiohttp


async def check_health(http_base: str) -> bool:
    try:
        async with aiohttp.ClientSession() as s:
            async with s.get(f"{http_base}/health", timeout=aiohttp.ClientTimeout(total=10)) as r:
                body = await r.json()
                print(f"health: HTTP {r.status} {json.dumps(body)}")
                return r.status == 200
    except Exception as e:  # pragma: no cover - manual tool
        print(f"health check failed: {e}")
        return False


async def run(url: str, messages, cfg) -> int:
    http_base = url.replace("ws://", "http://").replace("wss://", "https://").rsplit("/ws/", 1)[0]
    if not await check_health(http_base):
        return 1
    async with aiohttp.ClientSession() as s:
        async with s.ws_connect(url, max_msg_size=0) as ws:
            hello = json.loads((await ws.receive()).data)
            print(f"connected: {hello}")
            await ws.send_str(json.dumps({"type": "start_session", "config": cfg}))
            print(f"configured: {json.loads((await ws.receive()).data)}")
            interactive = not messages

            def next_message():
                if not interactive:
                    return messages.pop(0) if messages else None
                try:
                    return input("\nyou> ").strip() or None
                except EOFError:
                    return None

            while True:
                text = next_message()
                if text is None or text.lower() in ("quit", "exit"):
                    break
                await ws.send_str(json.dumps({"type": "user_message", "text": text}))
                t0 = time.perf_counter()
                first = None
                sys.stdout.write("assistant> ")
                while True:
                    msg = await ws.receive()
                    if msg.type != aiohttp.WSMsgType.TEXT:
                        print(f"\nconnection closed: {msg.type}")
                        return 1
                    f = json.loads(msg.data)
                    if f["type"] == "token":
                        if first is None:
                            first = time.perf_counter() - t0
                        sys.stdout.write(f["data"])
                        sys.stdout.flush()
                    elif f["type"] == "response_complete":
                        st = f["stats"]
                        print(f"\n[{st.get('tokens_generated')} tokens, "
                              f"{st.get('tokens_per_second', 0):.1f} tok/s, "
                              f"ttft {1e3 * (first or 0):.0f} ms client / "
                              f"{st.get('ttft_ms', 0):.0f} ms server]")
                        break
                    elif f["type"] == "error":
                        print(f"\nerror: {f['error']}")
                        break
            await ws.send_str(json.dumps({"type": "end_session"}))
            ended = json.loads((await ws.receive()).data)
            print(f"session ended: {json.dumps(ended.get('stats', {}))}")
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="ws://127.0.0.1:8000/ws/llm")
    ap.add_argument("-m", "--message", action="append", default=[])
    ap.add_argument("--system-prompt", default="You are a helpful voice assistant.")
    ap.add_argument("--temperature", type=float, default=0.7)
    ap.add_argument("--max-tokens", type=int, default=128)
    a = ap.parse_args()
    cfg = {"system_prompt": a.system_prompt, "temperature": a.temperature, "max_tokens": a.max_tokens}
    return asyncio.run(run(a.url, list(a.message), cfg))


if __name__ == "__main__":
    sys.exit(main())
