"""aiohttp application factory.

``make_app(state)`` registers every route whose backing component exists on
``state``; the full control plane (jobs, workers, dashboard, debug, costs,
...) is wired by ``llm_mcp_amd.api.routes`` when a store is configured."""
from __future__ import annotations

from aiohttp import web

from ..utils import tracing
from .helpers import write_error, write_json
from .openai_chat import ChatHandler


class ServingState:
    """Minimal state: the local model registry + metrics (the serving slice)."""

    def __init__(self, registry, metrics, version: str = "0.1.0", circuit=None):
        self.registry = registry
        self.metrics = metrics
        self.version = version
        self.circuit = circuit


STATE_KEY = web.AppKey("state", object)


def make_app(state) -> web.Application:
    app = web.Application(client_max_size=10 << 20, middlewares=[tracing.aiohttp_middleware()])
    app[STATE_KEY] = state
    chat_handler = ChatHandler(state)

    async def chat(request):
        return await chat_handler(request)

    async def health(request):
        return write_json(200, {"status": "ok", "version": state.version})

    async def metrics(request):
        return web.Response(body=state.metrics.render(),
                            headers={"Content-Type": "text/plain; version=0.0.4"})

    async def trace(request):
        """Spans recorded in this process for one request ID."""
        if request.method != "GET":
            return write_error(405, "method_not_allowed", "Method not allowed")
        rid = tracing.clean_id(request.match_info.get("rid", ""))
        spans = tracing.RING.find(rid) if rid else []
        if not spans:
            return write_error(404, "not_found", "No spans recorded for this request id")
        return write_json(200, {"request_id": rid, "spans": spans})

    app.router.add_route("*", "/v1/debug/trace/{rid}", trace)
    app.router.add_route("*", "/health", health)
    app.router.add_route("*", "/version", health)
    app.router.add_route("GET", "/metrics", metrics)
    app.router.add_route("*", "/v1/chat/completions", chat)
    extra = getattr(state, "register_routes", None)
    if extra is not None:
        extra(app)
    return app
