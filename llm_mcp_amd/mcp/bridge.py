"""HTTP bridge (default :3333), reference: mcp/src/index.ts.

Routes: GET /health; POST /submit (gRPC SubmitJob); GET /jobs/{id} (gRPC
GetJob); GET /jobs/{id}/stream (gRPC StreamJob -> SSE ``event:<type>`` /
``data:<data_json>``); HTTP proxies /llm/request, /dashboard, /costs/summary,
/benchmarks, /discovery, /costs/balance, /models/stats, /feedback,
/knowledge/ingest, /models/sync; plus /chat/completions and /embeddings.
Fixed defects: /discovery targets the existing /v1/discovery/last route
(the reference proxied to a nonexistent /v1/discovery), and /submit without
a ``kind`` but with model/prompt creates an engine.generate job (the
reference silently created echo jobs, fastmcp/server.py:55-69).
"""
from __future__ import annotations

import asyncio
import json
import os

from aiohttp import ClientSession, ClientTimeout, web

from ..api.helpers import write_error, write_json

PROXIES = {
    ("POST", "/llm/request"): "/v1/llm/request",
    ("GET", "/dashboard"): "/v1/dashboard",
    ("GET", "/costs/summary"): "/v1/costs/summary",
    ("GET", "/benchmarks"): "/v1/benchmarks",
    ("GET", "/discovery"): "/v1/discovery/last",
    ("POST", "/discovery/run"): "/v1/discovery/run",
    ("GET", "/costs/balance"): "/v1/costs/balance",
    ("GET", "/models/stats"): "/v1/models/stats",
    ("POST", "/feedback"): "/v1/feedback",
    ("POST", "/knowledge/ingest"): "/v1/knowledge/ingest",
    ("POST", "/models/sync"): "/v1/models/sync",
    ("POST", "/chat/completions"): "/v1/chat/completions",
    ("POST", "/embeddings"): "/v1/embeddings",
}


def submit_request(body: dict) -> tuple[str, dict, int]:
    kind = body.get("kind") or ""
    payload = body.get("payload")
    if not kind and (body.get("prompt") or body.get("messages")):
        kind = "engine.generate"
        payload = {k: body[k] for k in ("model", "prompt", "messages", "device_id", "thinking")
                   if body.get(k) is not None}
        opts = {k: body[k] for k in ("temperature", "max_tokens", "top_p", "top_k", "stop")
                if body.get(k) is not None}
        if body.get("system"):
            payload["messages"] = [{"role": "system", "content": body["system"]},
                                   {"role": "user", "content": body.get("prompt", "")}]
        if body.get("device") and "device_id" not in payload:
            payload["device_id"] = body["device"]
        if opts:
            payload["options"] = opts
    return kind or "echo", payload if isinstance(payload, dict) else {}, int(body.get("priority", 0))


def make_bridge(core_http: str, grpc_client) -> web.Application:
    app = web.Application()
    core_http = core_http.rstrip("/")

    async def health(request):
        return write_json(200, {"status": "ok"})

    async def submit(request):
        try:
            body = await request.json()
        except Exception:
            return write_error(400, "invalid_json", "Invalid JSON body")
        kind, payload, prio = submit_request(body)
        try:
            jid = await asyncio.to_thread(grpc_client.submit, kind, payload, prio, "mcp")
        except Exception as e:
            return write_error(502, "core_unavailable", str(e))
        return write_json(202, {"job_id": jid, "kind": kind})

    async def job(request):
        jid = request.match_info["jid"]
        try:
            j = await asyncio.to_thread(grpc_client.get, jid)
        except Exception as e:
            return write_error(404, "not_found", str(e))
        return write_json(200, j)

    async def job_stream(request):
        jid = request.match_info["jid"]
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream",
                                           "Cache-Control": "no-cache"})
        await resp.prepare(request)
        q: asyncio.Queue = asyncio.Queue()
        loop = asyncio.get_running_loop()

        def pump():
            try:
                for ev in grpc_client.stream(jid):
                    loop.call_soon_threadsafe(q.put_nowait, ev)
            except Exception as e:
                loop.call_soon_threadsafe(q.put_nowait, {"type": "error",
                                                         "data": {"error": str(e)}})
            loop.call_soon_threadsafe(q.put_nowait, None)

        threading_task = asyncio.get_running_loop().run_in_executor(None, pump)
        while True:
            ev = await q.get()
            if ev is None:
                break
            await resp.write(f"event: {ev['type']}\ndata: {json.dumps(ev['data'])}\n\n".encode())
        await threading_task
        return resp

    async def proxy(request):
        target = PROXIES.get((request.method, request.path))
        if target is None:
            return write_error(404, "not_found", "Resource not found")
        qs = ("?" + request.query_string) if request.query_string else ""
        body = await request.read()
        try:
            async with ClientSession(timeout=ClientTimeout(total=180)) as s:
                async with s.request(request.method, core_http + target + qs, data=body or None,
                                     headers={"Content-Type": "application/json"}) as r:
                    ct = r.headers.get("Content-Type", "application/json")
                    if ct.startswith("text/event-stream"):
                        out = web.StreamResponse(status=r.status, headers={"Content-Type": ct})
                        await out.prepare(request)
                        async for chunk in r.content.iter_any():
                            await out.write(chunk)
                        return out
                    return web.Response(status=r.status, body=await r.read(),
                                        headers={"Content-Type": ct})
        except Exception as e:
            return write_error(502, "core_unavailable", str(e))

    app.router.add_get("/health", health)
    app.router.add_post("/submit", submit)
    app.router.add_get("/jobs/{jid}/stream", job_stream)
    app.router.add_get("/jobs/{jid}", job)
    for (m, p) in PROXIES:
        app.router.add_route(m, p, proxy)
    return app


def main():
    from ..rpc.client import CoreClient
    addr = os.environ.get("MCP_HTTP_ADDR", "0.0.0.0:3333")
    host, port = addr.rsplit(":", 1)
    app = make_bridge(os.environ.get("CORE_HTTP_URL", "http://127.0.0.1:8080"),
                      CoreClient(os.environ.get("CORE_GRPC_ADDR", "127.0.0.1:9090")))
    web.run_app(app, host=host or "0.0.0.0", port=int(port), access_log=None)


if __name__ == "__main__":
    main()
