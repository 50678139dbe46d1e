"""``python -m llm_mcp_amd.api.serve`` -- the API ("core") process.

Serves the OpenAI-compatible endpoints (and, with a store configured, the
whole control plane) and forwards generation to engine worker processes over
their Unix sockets (engine/ipc.py).  Engines are given as
``--engine MODEL=unix:/path[,device=gpu0]`` (repeatable); the process keeps
retrying until every engine socket is up, and ``GET /ready`` turns 200 once
all are connected (``/health`` answers immediately, as in the reference).

Engine links are supervised: when a worker process dies its replicas leave
the registry (new requests route to the survivors, its in-flight streams end
with ``finish_reason: "error"``) and the link re-attaches as soon as a
replacement worker opens the socket again -- the in-process form of the
reference's restartable worker units (compose.yml:117,133,149
``restart: unless-stopped``).

Several API processes can share one port (``--reuse-port``, SO_REUSEPORT):
the kernel spreads client connections over them, so one event loop does not
bound the node's SSE rate, and with ``--shared-load`` they select replicas on
node-wide in-flight counts (api/shared_load.py) -- bench.py runs the front
door this way.
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

LIVE_INFO_S = float(os.environ.get("LMX_ENGINE_INFO_S", "5"))


def parse_engine_spec(spec: str) -> dict:
    model, rest = spec.split("=", 1)
    parts = rest.split(",")
    out = {"model": model, "path": parts[0].removeprefix("unix:"), "device": "gpu0"}
    for p in parts[1:]:
        k, v = p.split("=", 1)
        out[k] = v
    return out


async def _link(state, s: dict, first: asyncio.Future, supervise: bool) -> None:
    """One engine link: connect, register the replica, keep its live info
    (KV usage, running / waiting, step stats) fresh, and on disconnect drop
    the replica and re-attach when the socket comes back."""
    cfg = mc.resolve(s["model"])
    tok = for_model(cfg, s.get("tokenizer"))
    while True:
        c = EngineClient(s["path"])
        await c.connect()
        try:
            info = await c.info(timeout=30)
        except (ConnectionError, asyncio.TimeoutError) as e:
            log.warning("engine %s on %s: info failed (%s); retrying", s["model"], s["path"], e)
            await c.close()
            await asyncio.sleep(0.5)
            continue
        minfo = {**info, **(info.get("models") or {}).get(s["model"], {})}
        lm = LocalModel(
            s["model"], minfo.get("kind", "chat"),
            s.get("device") or minfo.get("device_id", "gpu0"), c, tok, cfg,
            max_model_len=int(minfo.get("max_model_len", 8192)),
            capacity=int(minfo.get("capacity", 256)),
            tags={"tp_comm": minfo.get("tp_comm") or {}, "live": info},
            lb_slot=int(s.get("slot", -1)))
        state.registry.add(lm)
        log.info("engine %s on %s connected (%s)", s["model"], s["path"], lm.device_id)
        if not first.done():
            first.set_result(True)

        async def poll():
            while c.connected.is_set():
                await asyncio.sleep(LIVE_INFO_S)
                try:
                    lm.tags["live"] = await c.info(timeout=LIVE_INFO_S)
                except (ConnectionError, asyncio.TimeoutError, RuntimeError):
                    pass

        poller = asyncio.create_task(poll())
        await c.wait_closed()
        poller.cancel()
        state.registry.remove(lm)
        log.error("engine %s on %s (%s) disconnected; replica removed", s["model"],
                  s["path"], lm.device_id)
        if not supervise:
            return
        await asyncio.sleep(0.5)


async def attach_engines(state, specs: list[dict], supervise: bool = True):
    """Attach every engine; returns once each has connected once (then
    ``state.engines_ready``).  The link tasks stay alive on
    ``state.engine_links`` and re-attach restarted workers."""
    loop = asyncio.get_running_loop()
    for i, s in enumerate(specs):
        s.setdefault("slot", i)           # column in a shared front-door load table
    firsts = [loop.create_future() for _ in specs]
    links = [asyncio.create_task(_link(state, s, f, supervise)) for s, f in zip(specs, firsts)]
    state.engine_links = getattr(state, "engine_links", []) + links
    if firsts:
        await asyncio.gather(*firsts)
    state.engines_ready = True


def make_serving_app(specs: list[dict], version: str | None = None, ready_file: str = "",
                     shared_load: tuple[str, int, int] | None = None):
    """The API process's app: chat + embeddings + /ready over attached
    engine sockets (attached on startup).  ``shared_load`` = (path, index,
    count): this is API process ``index`` of ``count`` sharing one port, and
    replica selection balances on the node-wide counts (api/shared_load.py)."""
    state = ServingState(ModelRegistry(), Metrics(),
                         version=version or os.environ.get("CORE_VERSION", "0.1.0"),
                         circuit=CircuitBreaker())
    state.engines_ready = False
    if shared_load is not None:
        from .shared_load import SharedLoad
        path, index, count = shared_load
        state.registry.balancer = SharedLoad(path, index, count, max(1, len(specs)))

    def register(app):
        async def ready(request):
            ok = getattr(state, "engines_ready", False)
            return write_json(200 if ok else 503, {"ready": ok,
                                                    "models": state.registry.model_ids(),
                                                    "replicas": len(state.registry.all())})
        app.router.add_get("/ready", ready)
        emb = EmbeddingsHandler(state)

        async def embeddings(request):
            return await emb(request)
        app.router.add_route("*", "/v1/embeddings", embeddings)

    state.register_routes = register
    app = make_app(state)

    async def attach():
        await attach_engines(state, specs)
        if ready_file:
            with open(ready_file, "w") as f:
                f.write(str(os.getpid()))

    async def on_start(app):
        app[_ATTACH] = asyncio.create_task(attach())

    async def on_cleanup(app):
        for t in getattr(state, "engine_links", []):
            t.cancel()

    app.on_startup.append(on_start)
    app.on_cleanup.append(on_cleanup)
    return app, state


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default=os.environ.get("LMX_HTTP_HOST", "127.0.0.1"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("LMX_HTTP_PORT", "8080")))
    ap.add_argument("--engine", action="append", default=[],
                    help="MODEL=unix:/path[,device=gpu0][,tokenizer=/dir]")
    ap.add_argument("--reuse-port", action="store_true",
                    help="SO_REUSEPORT: several API processes serve one port")
    ap.add_argument("--ready-file", default="",
                    help="written once every engine is attached")
    ap.add_argument("--shared-load", default="",
                    help="/dev/shm file of node-wide in-flight counts shared by the API "
                         "processes of one port (with --api-index / --api-count)")
    ap.add_argument("--api-index", type=int, default=0)
    ap.add_argument("--api-count", type=int, default=1)
    a = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("LOG_LEVEL", "INFO"))
    shared = (a.shared_load, a.api_index, a.api_count) if a.shared_load else None
    app, _ = make_serving_app([parse_engine_spec(s) for s in a.engine], ready_file=a.ready_file,
                              shared_load=shared)
    web.run_app(app, host=a.host, port=a.port, access_log=None, print=None,
                reuse_port=a.reuse_port or None)


if __name__ == "__main__":
    main()
