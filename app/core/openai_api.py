"""OpenAI-compatible facade over the in-process engine (E1): ``GET /v1/models``,
``POST /v1/chat/completions`` (``stream`` via SSE, ``tools`` with server-side
hermes / llama3_json parsing like vLLM's ``--enable-auto-tool-choice``,
``tool_choice="required"`` or a named function -> JSON-schema guided decoding),
``GET /health`` is on the main app.  Existing OpenAI/vLLM clients -- including
the reference's ``VLLMHandler`` / pydantic-ai agent -- can point their
``base_url`` at ``http://host:8000/v1``.
"""
from __future__ import annotations

import json
import time
import uuid
from typing import Any, Dict, List

from fastapi import Request
from fastapi.responses import JSONResponse, StreamingResponse


def register_openai_routes(app, handler) -> None:
    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": handler.model, "object": "model",
                                             "created": int(time.time()), "owned_by": "fasttalk"}]}

    @app.post("/v1/chat/completions")
    async def chat_completions(request: Request):
        from fasttalk_llm_microservice_amd.engine.guided import GuidedSpec
        from fasttalk_llm_microservice_amd.engine.tool_parser import (StreamingToolCallParser,
                                                                       StreamingToolDetector,
                                                                       parse_tool_calls)

        try:
            body = await request.json()
        except Exception:
            return JSONResponse({"error": {"message": "invalid JSON body"}}, status_code=400)
        messages: List[Dict[str, Any]] = body.get("messages") or []
        if not messages:
            return JSONResponse({"error": {"message": "messages is required"}}, status_code=400)
        tools = body.get("tools") or None
        tool_choice = body.get("tool_choice", "auto")
        guided = None
        if tools and (tool_choice == "required" or isinstance(tool_choice, dict)):
            pick = tools
            if isinstance(tool_choice, dict):
                name = (tool_choice.get("function") or {}).get("name")
                pick = [t for t in tools if (t.get("function") or t).get("name") == name] or tools
            guided = GuidedSpec.tool_call(pick)
        rf = body.get("response_format") or {}
        if guided is None and rf.get("type") == "json_schema":
            guided = GuidedSpec.json_schema((rf.get("json_schema") or {}).get("schema") or {})
        stop = body.get("stop")
        if isinstance(stop, str):
            stop = [stop]
        kw = dict(temperature=body.get("temperature", 1.0), max_tokens=body.get("max_tokens")
                  or body.get("max_completion_tokens"), top_p=body.get("top_p"),
                  top_k=body.get("top_k"), stop=stop, tools=tools, guided=guided,
                  seed=body.get("seed"), ignore_eos=bool(body.get("ignore_eos", False)),
                  min_tokens=int(body.get("min_tokens") or 0))
        rid = f"chatcmpl-{uuid.uuid4().hex[:24]}"
        created = int(time.time())
        model = body.get("model") or handler.model

        def chunk(delta: Dict[str, Any], finish=None) -> str:
            return "data: " + json.dumps({"id": rid, "object": "chat.completion.chunk",
                                          "created": created, "model": model,
                                          "choices": [{"index": 0, "delta": delta,
                                                       "finish_reason": finish}]}) + "\n\n"

        if body.get("stream"):
            async def gen():
                """With ``tools``, the first visible characters decide (like vLLM's
                auto tool choice): speech streams as ``content`` deltas at once; a
                tool call streams as ``tool_calls`` deltas -- id + name as soon as
                the name is complete, then argument fragments as they decode."""
                yield chunk({"role": "assistant", "content": ""})
                finish = "stop"
                det = StreamingToolDetector() if tools else None
                names = [(t.get("function") or t).get("name") for t in tools or []]
                tcp = StreamingToolCallParser(names) if tools else None
                any_call = False
                tool_text = []   # what the parser consumed, re-sent as content if no call
                async for out in handler.stream_events(messages, request_id=rid, **kw):
                    if out.finished:
                        finish = out.finish_reason
                    if not out.text:
                        continue
                    if det is None:
                        yield chunk({"content": out.text})
                        continue
                    mode, emit = det.feed(out.text)
                    if mode == "text":
                        if emit:
                            yield chunk({"content": emit})
                    elif mode == "tool":
                        held, det.buf = det.buf, ""   # the parser owns the tool text now
                        tool_text.append(held)
                        deltas = tcp.feed(held)
                        if deltas:
                            any_call = True
                            yield chunk({"tool_calls": deltas})
                if det is not None and det.mode is None and det.buf:
                    yield chunk({"content": det.buf})   # never became a tool call
                elif det is not None and det.mode == "tool" and not any_call and tool_text:
                    # looked like a call ('{', a tag) but no call of a requested tool
                    # came out of it: it was text (e.g. a JSON answer)
                    yield chunk({"content": "".join(tool_text)})
                if any_call:
                    finish = "tool_calls"
                yield chunk({}, finish if finish in ("stop", "length", "tool_calls") else "stop")
                yield "data: [DONE]\n\n"

            return StreamingResponse(gen(), media_type="text/event-stream")

        parts: List[str] = []
        n_prompt = n_out = 0
        finish = "stop"
        async for out in handler.stream_events(messages, request_id=rid, **kw):
            parts.append(out.text)
            n_out += len(out.token_ids)
            n_prompt = out.num_prompt_tokens or n_prompt
            if out.finished:
                finish = out.finish_reason
        text = "".join(parts)
        msg: Dict[str, Any] = {"role": "assistant", "content": text}
        if tools:
            calls, rest = parse_tool_calls(text)
            names = {(t.get("function") or t).get("name") for t in tools}
            if calls and all(c.name in names for c in calls):
                msg = {"role": "assistant", "content": rest or None,
                       "tool_calls": [c.to_openai() for c in calls]}
                finish = "tool_calls"
        return {"id": rid, "object": "chat.completion", "created": created, "model": model,
                "choices": [{"index": 0, "message": msg,
                             "finish_reason": finish if finish in ("stop", "length", "tool_calls") else "stop"}],
                "usage": {"prompt_tokens": n_prompt, "completion_tokens": n_out,
                          "total_tokens": n_prompt + n_out}}
