"""Agent tools (E17): ``duckduckgo_search`` (same tool name / argument schema as
pydantic-ai's ``duckduckgo_search_tool``, reference ``app/agents/voice_agent.py:
147-152``), ``get_current_time`` and ``get_session_info`` (``:173-188``).

There is no network in this environment, so the search tool has two backends:
``stub`` (default; deterministic offline results, BASELINE config 5 "web-search
stub") and ``duckduckgo`` (the DuckDuckGo HTML endpoint over httpx, used only
when ``WEB_SEARCH_BACKEND=duckduckgo``), rate-limited by
``DUCKDUCKGO_RATE_LIMIT`` seconds between calls.
"""
from __future__ import annotations

import asyncio
import hashlib
import html
import inspect
import os
import re
import time
from dataclasses import dataclass, field
from datetime import datetime
from typing import Any, Awaitable, Callable, Dict, List, Optional


@dataclass
class Tool:
    name: str
    description: str
    parameters: Dict[str, Any]
    fn: Callable[..., Any]
    takes_ctx: bool = True

    def schema(self) -> Dict[str, Any]:
        return {"type": "function", "function": {"name": self.name, "description": self.description,
                                                 "parameters": self.parameters}}

    async def __call__(self, ctx, **kwargs) -> str:
        res = self.fn(ctx, **kwargs) if self.takes_ctx else self.fn(**kwargs)
        if inspect.isawaitable(res):
            res = await res
        return res if isinstance(res, str) else str(res)


class _RateLimiter:
    def __init__(self, interval: float):
        self.interval = max(0.0, interval)
        self._last = 0.0
        self._lock = asyncio.Lock()

    async def wait(self):
        async with self._lock:
            dt = time.monotonic() - self._last
            if dt < self.interval:
                await asyncio.sleep(self.interval - dt)
            self._last = time.monotonic()


def _stub_results(query: str, max_results: int) -> List[Dict[str, str]]:
    h = hashlib.sha1(query.encode()).hexdigest()
    return [{
        "title": f"{query.strip().title()} - result {i + 1}",
        "href": f"https://example.org/{h[:8]}/{i + 1}",
        "body": f"Offline search stub: summary {i + 1} for '{query.strip()}' (ref {h[i:i + 6]}).",
    } for i in range(max_results)]


async def _duckduckgo_html(query: str, max_results: int) -> List[Dict[str, str]]:
    import httpx

    async with httpx.AsyncClient(timeout=10.0, follow_redirects=True) as c:
        r = await c.post("https://html.duckduckgo.com/html/", data={"q": query},
                         headers={"User-Agent": "fasttalk-mi355x/1.0"})
        r.raise_for_status()
    out = []
    for m in re.finditer(r'class="result__a" href="([^"]+)"[^>]*>(.*?)</a>.*?class="result__snippet"[^>]*>(.*?)</',
                         r.text, re.S):
        strip = lambda s: html.unescape(re.sub(r"<[^>]+>", "", s)).strip()  # noqa: E731
        out.append({"title": strip(m.group(2)), "href": m.group(1), "body": strip(m.group(3))})
        if len(out) >= max_results:
            break
    return out


def make_search_tool(rate_limit: float = 1.0, backend: Optional[str] = None) -> Tool:
    backend = (backend or os.getenv("WEB_SEARCH_BACKEND", "stub")).lower()
    limiter = _RateLimiter(rate_limit)

    async def duckduckgo_search(ctx, query: str, max_results: int = 5) -> str:
        max_results = max(1, min(int(max_results or 5), 10))
        if backend == "duckduckgo":
            await limiter.wait()  # only the live endpoint is rate limited
            try:
                results = await _duckduckgo_html(query, max_results)
            except Exception as e:  # offline or blocked: degrade to the stub
                results = _stub_results(query, max_results)
                results[0]["body"] += f" [live search unavailable: {type(e).__name__}]"
        else:
            results = _stub_results(query, max_results)
        import json

        return json.dumps(results)

    return Tool("duckduckgo_search",
                "Searches DuckDuckGo for the given query and returns the results.",
                {"type": "object", "properties": {
                    "query": {"type": "string", "description": "The query to search for."},
                    "max_results": {"type": "integer", "description": "The maximum number of results."}},
                 "required": ["query"]},
                duckduckgo_search)


def make_time_tool() -> Tool:
    def get_current_time(ctx) -> str:
        return f"The current date and time is {datetime.now().strftime('%A, %B %d, %Y at %I:%M %p')}."

    return Tool("get_current_time", "Get the current date and time.",
                {"type": "object", "properties": {}}, get_current_time)


def make_session_tool() -> Tool:
    def get_session_info(ctx) -> str:
        n = len(getattr(ctx, "conversation_history", []) or [])
        created = getattr(ctx, "created_at", datetime.now())
        dur = int((datetime.now() - created).total_seconds())
        sid = str(getattr(ctx, "session_id", "unknown"))
        return f"Session {sid[:8]}... has been active for {dur} seconds with {n} messages exchanged."

    return Tool("get_session_info", "Get information about the current conversation session.",
                {"type": "object", "properties": {}}, get_session_info)
