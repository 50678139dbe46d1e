"""MCP tool server -- native JSON-RPC 2.0 (no fastmcp dependency), stdio and
streamable-HTTP transports (reference: fastmcp/server.py, 12 tools).

Tools (reference names kept): llm_dashboard, llm_submit, llm_job_status,
llm_request, llm_costs, llm_benchmarks, llm_balance, llm_model_stats,
llm_feedback, llm_learn, llm_remember, llm_sync_models; added: llm_chat
(synchronous chat completion on the local GPUs), llm_embed, llm_capacity.
``llm_submit`` creates a real generation job (the reference's created echo
jobs).  Backend = the bridge (BACKEND_URL, default http://localhost:3333).
"""
from __future__ import annotations

import asyncio
import json
import os
import sys

import aiohttp

PROTOCOL_VERSION = "2025-03-26"


def _schema(props: dict, required: list[str]) -> dict:
    return {"type": "object", "properties": props, "required": required}


S, I, N = {"type": "string"}, {"type": "integer"}, {"type": "number"}
TOOLS = {
    "llm_dashboard": ("Full LLM panel: GPUs, engines, models, jobs, costs, hosts.",
                      _schema({}, []), ("GET", "/dashboard", None)),
    "llm_submit": ("Queue an LLM generation job; returns job_id.",
                   _schema({"model": S, "prompt": S, "system": S, "temperature": N,
                            "max_tokens": I, "device": S}, ["prompt"]),
                   ("POST", "/submit", None)),
    "llm_job_status": ("Status and result of a job.", _schema({"job_id": S}, ["job_id"]),
                       ("GET", "/jobs/{job_id}", None)),
    "llm_request": ("Routed LLM request (picks provider/model/GPU); returns job_id.",
                    _schema({"model": S, "prompt": S, "system": S, "temperature": N,
                             "max_tokens": I, "quality": S, "task": S}, ["prompt"]),
                    ("POST", "/llm/request", None)),
    "llm_costs": ("Spend summary per provider.", _schema({"period": S}, []),
                  ("GET", "/costs/summary", "period")),
    "llm_benchmarks": ("Model benchmark results per GPU.", _schema({}, []),
                       ("GET", "/benchmarks", None)),
    "llm_balance": ("Cloud balance and spend windows.", _schema({}, []),
                    ("GET", "/costs/balance", None)),
    "llm_model_stats": ("Per-model requests, tokens, cost, feedback.", _schema({}, []),
                        ("GET", "/models/stats", None)),
    "llm_feedback": ("Rate a model answer: good | bad.",
                     _schema({"model": S, "rating": S, "comment": S}, ["model", "rating"]),
                     ("POST", "/feedback", None)),
    "llm_learn": ("Store knowledge in LightRAG (>= 100 chars).",
                  _schema({"text": S, "topic": S, "domain": S}, ["text", "topic"]),
                  ("POST", "/knowledge/ingest", "learn")),
    "llm_remember": ("Store a fact / preference in mem0.",
                     _schema({"text": S, "user_id": S}, ["text"]),
                     ("POST", "/knowledge/ingest", "remember")),
    "llm_sync_models": ("Refresh the model catalogue.", _schema({}, []),
                        ("POST", "/models/sync", None)),
    "llm_chat": ("Synchronous chat completion on the local MI355X engines.",
                 _schema({"model": S, "prompt": S, "system": S, "temperature": N,
                          "max_tokens": I}, ["prompt"]),
                 ("POST", "/chat/completions", "chat")),
    "llm_embed": ("Embeddings on the local GPUs.",
                  _schema({"model": S, "input": S, "dimensions": I}, ["input"]),
                  ("POST", "/embeddings", "embed")),
}


def build_call(name: str, args: dict) -> tuple[str, str, dict | None, dict | None]:
    desc, _schema_, (method, path, mode) = TOOLS[name]
    params = None
    body = None
    if "{job_id}" in path:
        path = path.replace("{job_id}", str(args["job_id"]))
    if method == "GET":
        if mode == "period":
            params = {"period": args.get("period", "day")}
        return method, path, None, params
    if mode == "learn":
        body = {"text": args["text"], "target": "lightrag",
                "metadata": {"source_type": "agent-learning", "topic": args.get("topic", ""),
                             "domain": args.get("domain", "General")}}
    elif mode == "remember":
        body = {"text": args["text"], "target": "mem0", "user_id": args.get("user_id", "default")}
    elif mode == "chat":
        msgs = ([{"role": "system", "content": args["system"]}] if args.get("system") else []) + \
            [{"role": "user", "content": args["prompt"]}]
        body = {"model": args.get("model") or os.environ.get("LMX_CHAT_MODEL", "llama-3-8b"),
                "messages": msgs, "temperature": args.get("temperature", 0.7),
                "max_tokens": args.get("max_tokens", 512)}
    elif mode == "embed":
        body = {"model": args.get("model") or os.environ.get("LMX_EMBED_MODEL",
                                                             "nomic-embed-text"),
                "input": args["input"]}
        if args.get("dimensions"):
            body["dimensions"] = args["dimensions"]
    else:
        body = dict(args)
    return method, path, body, params


class MCPServer:
    def __init__(self, backend: str | None = None):
        self.backend = (backend or os.environ.get("BACKEND_URL", "http://localhost:3333")).rstrip("/")
        self._session: aiohttp.ClientSession | None = None

    async def session(self):
        if self._session is None:
            self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=120))
        return self._session

    async def call_tool(self, name: str, args: dict) -> str:
        method, path, body, params = build_call(name, args or {})
        s = await self.session()
        async with s.request(method, self.backend + path, json=body, params=params) as r:
            text = await r.text()
            if r.status >= 400:
                raise RuntimeError(f"HTTP {r.status}: {text[:500]}")
            return text

    async def handle(self, msg: dict) -> dict | None:
        mid = msg.get("id")
        method = msg.get("method", "")
        if mid is None:  # notification
            return None
        try:
            if method == "initialize":
                res = {"protocolVersion": PROTOCOL_VERSION,
                       "capabilities": {"tools": {"listChanged": False}},
                       "serverInfo": {"name": "llm", "version": "1.0"}}
            elif method == "ping":
                res = {}
            elif method == "tools/list":
                res = {"tools": [{"name": n, "description": d, "inputSchema": sc}
                                 for n, (d, sc, _) in TOOLS.items()]}
            elif method == "tools/call":
                p = msg.get("params") or {}
                name = p.get("name")
                if name not in TOOLS:
                    return {"jsonrpc": "2.0", "id": mid,
                            "error": {"code": -32602, "message": f"unknown tool {name}"}}
                try:
                    text = await self.call_tool(name, p.get("arguments") or {})
                    res = {"content": [{"type": "text", "text": text}], "isError": False}
                except Exception as e:
                    res = {"content": [{"type": "text", "text": str(e)}], "isError": True}
            else:
                return {"jsonrpc": "2.0", "id": mid,
                        "error": {"code": -32601, "message": f"method not found: {method}"}}
        except Exception as e:
            return {"jsonrpc": "2.0", "id": mid, "error": {"code": -32603, "message": str(e)}}
        return {"jsonrpc": "2.0", "id": mid, "result": res}

    async def serve_stdio(self, reader=None, writer=None):
        loop = asyncio.get_running_loop()
        inp = reader or sys.stdin
        out = writer or sys.stdout
        while True:
            line = await loop.run_in_executor(None, inp.readline)
            if not line:
                break
            line = line.strip()
            if not line:
                continue
            try:
                msg = json.loads(line)
            except ValueError:
                out.write(json.dumps({"jsonrpc": "2.0", "id": None,
                                      "error": {"code": -32700, "message": "parse error"}}) + "\n")
                out.flush()
                continue
            msgs = msg if isinstance(msg, list) else [msg]
            for m in msgs:
                r = await self.handle(m)
                if r is not None:
                    out.write(json.dumps(r) + "\n")
                    out.flush()

    def http_app(self):
        from aiohttp import web

        async def rpc(request):
            body = await request.json()
            msgs = body if isinstance(body, list) else [body]
            res = [r for r in [await self.handle(m) for m in msgs] if r is not None]
            if not res:
                return web.Response(status=202)
            return web.json_response(res if isinstance(body, list) else res[0])
        app = web.Application()
        app.router.add_post("/mcp", rpc)
        return app


def main():
    srv = MCPServer()
    if "--http" in sys.argv:
        from aiohttp import web
        web.run_app(srv.http_app(), port=int(os.environ.get("MCP_PORT", "8765")))
    else:
        asyncio.run(srv.serve_stdio())


if __name__ == "__main__":
    main()
