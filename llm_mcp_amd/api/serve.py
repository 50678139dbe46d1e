"""``python -m llm_mcp_amd.api.serve`` -- the API ("core") process.

Serves the OpenAI-compatible endpoints (and, with a store configured, the
whole control plane) and forwards generation to engine worker processes over
their Unix sockets (engine/ipc.py).  Engines are given as
``--engine MODEL=unix:/path[,device=gpu0]`` (repeatable); the process keeps
retrying until every engine socket is up, and ``GET /ready`` turns 200 once
all are connected (``/health`` answers immediately, as in the reference).
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os

from aiohttp import web

from ..engine.ipc import EngineClient
from ..models import config as mc
from ..models.tokenizer import for_model
from ..utils.metrics import Metrics
from ..policy.circuit import CircuitBreaker
from .app import ServingState, make_app
from .helpers import write_json
from .openai_embed import EmbeddingsHandler
from .registry import LocalModel, ModelRegistry

log = logging.getLogger("lmx.serve")
_ATTACH = web.AppKey("attach", asyncio.Task)


def parse_engine_spec(spec: str) -> dict:
    model, rest = spec.split("=", 1)
    parts = rest.split(",")
    out = {"model": model, "path": parts[0].removeprefix("unix:"), "device": "gpu0"}
    for p in parts[1:]:
        k, v = p.split("=", 1)
        out[k] = v
    return out


async def attach_engines(state, specs: list[dict]):
    clients = []
    for s in specs:
        c = EngineClient(s["path"])
        clients.append((s, c))

    async def one(s, c):
        await c.connect()
        info = await c.info(timeout=30)
        info = {**info, **(info.get("models") or {}).get(s["model"], {})}
        cfg = mc.resolve(s["model"])
        state.registry.add(LocalModel(
            s["model"], info.get("kind", "chat"), s.get("device") or info.get("device_id", "gpu0"),
            c, for_model(cfg, s.get("tokenizer")), cfg,
            max_model_len=int(info.get("max_model_len", 8192)),
            capacity=int(info.get("capacity", 256)),
            tags={"tp_comm": info.get("tp_comm") or {}}))
        log.info("engine %s on %s connected", s["model"], s["path"])

    await asyncio.gather(*[one(s, c) for s, c in clients])
    state.engines_ready = True


def make_serving_app(specs: list[dict], version: str | None = None):
    """The API process's app: chat + embeddings + /ready over attached
    engine sockets (attached on startup)."""
    state = ServingState(ModelRegistry(), Metrics(),
                         version=version or os.environ.get("CORE_VERSION", "0.1.0"),
                         circuit=CircuitBreaker())
    state.engines_ready = False

    def register(app):
        async def ready(request):
            ok = getattr(state, "engines_ready", False)
            return write_json(200 if ok else 503, {"ready": ok,
                                                    "models": state.registry.model_ids()})
        app.router.add_get("/ready", ready)
        emb = EmbeddingsHandler(state)

        async def embeddings(request):
            return await emb(request)
        app.router.add_route("*", "/v1/embeddings", embeddings)

    state.register_routes = register
    app = make_app(state)

    async def on_start(app):
        app[_ATTACH] = asyncio.create_task(attach_engines(state, specs))

    app.on_startup.append(on_start)
    return app, state


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default=os.environ.get("LMX_HTTP_HOST", "127.0.0.1"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("LMX_HTTP_PORT", "8080")))
    ap.add_argument("--engine", action="append", default=[],
                    help="MODEL=unix:/path[,device=gpu0][,tokenizer=/dir]")
    a = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("LOG_LEVEL", "INFO"))
    app, _ = make_serving_app([parse_engine_spec(s) for s in a.engine])
    web.run_app(app, host=a.host, port=a.port, access_log=None, print=None)


if __name__ == "__main__":
    main()
