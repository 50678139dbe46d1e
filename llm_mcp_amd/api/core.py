"""The core process: HTTP API + control plane + background loops.

Replaces core/cmd/core/main.go:26-123: env config, store, migrations (the
store applies its schema idempotently at start -- the reference left
migrations 02-05 to be applied by hand), discovery, router, device limits
(+ ticker), deadline expiry + job retention (the documented-but-missing
planner), gRPC server, graceful shutdown of HTTP *and* gRPC.
"""
from __future__ import annotations

import asyncio
import atexit
import threading
import weakref
import logging
import os
import time

from aiohttp import web

from ..devices.discovery import DiscoveryRunner
from ..policy import limits as lim
from ..policy.circuit import CircuitBreaker
from ..policy.router import Router
from ..utils.metrics import Metrics
from .app import make_app
from .helpers import write_json
from .registry import ModelRegistry
from .routes import ControlPlane
from .selection import select_model

log = logging.getLogger("lmx.core")


def env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


def open_store(spec: str | None = None):
    """LMX_STORE = memory[:journal_path] | postgres (uses DB_DSN)."""
    spec = spec or os.environ.get("LMX_STORE", "memory")
    if spec.startswith("postgres") or (spec == "auto" and os.environ.get("DB_DSN")):
        from ..store.postgres import PostgresStore
        return PostgresStore(os.environ["DB_DSN"])
    from ..store.memory import MemoryStore
    journal = spec.split(":", 1)[1] if ":" in spec else os.environ.get("LMX_JOURNAL", "")
    return MemoryStore(journal_path=journal,
                       snapshot_path=os.environ.get("LMX_SNAPSHOT", ""))


class JobChangeHub:
    """One thread blocks in the store's change wait (native condition
    variable, or Postgres LISTEN) and wakes every asyncio waiter of the loop
    through one shared future.  A job SSE stream, a gRPC StreamJob or a
    claim long-poll awaiting a change then costs no thread: with one
    ``to_thread`` per waiter, 256 streams contended for the 32-thread default
    executor and every store change cycled all of them through it -- the
    config-5 core spent its CPU handing threads around (profiles/r6_config5.md)."""

    def __init__(self, store, loop: asyncio.AbstractEventLoop):
        self.store, self.loop = store, loop
        self.ver = store.job_version()
        self._fut = loop.create_future()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="lmx-job-hub", daemon=True)
        self._thread.start()
        _HUBS.add(self)

    def _run(self):
        v = self.ver
        while not self._stop.is_set():
            try:
                v2 = self.store.wait_job_change(v, 0.25)
            except Exception:          # a store hiccup: retry after a pause
                self._stop.wait(0.5)
                continue
            if v2 != v:
                v = v2
                try:
                    self.loop.call_soon_threadsafe(self._notify, v2)
                except RuntimeError:    # the loop closed
                    return

    def _notify(self, v):
        self.ver = v
        fut, self._fut = self._fut, self.loop.create_future()
        if not fut.done():
            fut.set_result(v)

    async def wait(self, since, timeout_s: float):
        """The version after ``since`` changed, or the current one after
        ``timeout_s`` (the wait_job_change contract, without a thread)."""
        if self.ver != since:
            return self.ver
        try:
            await asyncio.wait_for(asyncio.shield(self._fut), timeout_s)
        except asyncio.TimeoutError:
            pass
        return self.ver

    def close(self):
        self._stop.set()
        _HUBS.discard(self)
        if self._thread is not threading.current_thread():
            self._thread.join(timeout=2.0)


# Hubs still open at interpreter exit are stopped first: a daemon thread left
# inside the native wait while the interpreter finalises aborts the process.
_HUBS: "weakref.WeakSet[JobChangeHub]" = weakref.WeakSet()


@atexit.register
def _close_hubs():
    for h in list(_HUBS):
        h.close()


class CoreState:
    def __init__(self, store=None, registry: ModelRegistry | None = None,
                 metrics: Metrics | None = None, circuit: CircuitBreaker | None = None,
                 version: str | None = None, engine_addrs: dict | None = None):
        self.version = version or os.environ.get("CORE_VERSION",
                                                 os.environ.get("LLM_MCP_VERSION", "0.1.0"))
        self.store = store if store is not None else open_store()
        self.registry = registry or ModelRegistry()
        self.metrics = metrics or Metrics()
        self.circuit = circuit or CircuitBreaker()
        self.router = Router(self.store, self.circuit, capacity_of=self._capacity_of)
        self.discovery = DiscoveryRunner(self.store, self.registry, self.metrics, engine_addrs)
        self.control = ControlPlane(self)
        self.engines_ready = True
        from .openai_embed import EmbeddingsHandler
        self.embed_handler = EmbeddingsHandler(self)
        self.cloud_embed = None
        self.cloud_chat = None
        self._tasks: list[asyncio.Task] = []
        self._hub: JobChangeHub | None = None

    def job_hub(self) -> JobChangeHub:
        """The change hub of the running loop (created on first use)."""
        loop = asyncio.get_running_loop()
        if self._hub is None or self._hub.loop is not loop:
            if self._hub is not None:
                self._hub.close()
            self._hub = JobChangeHub(self.store, loop)
        return self._hub

    def _capacity_of(self, device_id: str):
        caps = [m.capacity for m in self.registry.all() if m.device_id == device_id]
        return max(caps) if caps else None

    # chat-completions hooks ------------------------------------------------
    async def select_model(self, request, body: dict) -> str | None:
        task = request.headers.get("X-Task-Type") or body.get("task_type") or "general"
        acc = request.headers.get("X-Accuracy") or body.get("accuracy") or "medium"
        max_cost = float(body.get("max_cost_usd") or 0)
        if request.headers.get("X-Max-Cost"):
            try:
                max_cost = float(request.headers["X-Max-Cost"])
            except ValueError:
                pass
        local = [{"id": m.model_id, "context_k": m.max_model_len // 1024}
                 for m in self.registry.all() if m.kind == "chat"]
        return select_model(self.store.list_model_rankings(), local, task, acc, max_cost,
                            body.get("messages") or [])

    def on_chat_done(self, model: str, n_in: int, n_out: int, ms: int, status: str):
        try:
            cost = self.store.calculate_job_cost(model, n_in, n_out)
            self.store.update_model_stats(model, n_in, n_out, ms, cost, status != "error")
            if cost:
                self.store.insert_cost(None, model, "local", n_in, n_out, cost)
        except Exception:
            log.exception("model stats update failed")

    # routes ------------------------------------------------------------------
    def register_routes(self, app: web.Application):
        self.control.register(app)

        async def ready(request):
            return write_json(200 if self.engines_ready else 503,
                              {"ready": self.engines_ready, "models": self.registry.model_ids(),
                               "replicas": len(self.registry.all())})
        app.router.add_get("/ready", ready)
        if self.embed_handler is not None:
            h = self.embed_handler

            async def emb(request):
                return await h(request)
            app.router.add_route("*", "/v1/embeddings", emb)

    # background loops ----------------------------------------------------------
    async def _every(self, seconds: float, fn, name: str):
        while True:
            try:
                await asyncio.to_thread(fn)
            except Exception:
                log.exception("%s failed", name)
            await asyncio.sleep(seconds)

    def _maintenance(self):
        from ..planner.catalog import RetentionPlanner
        if not hasattr(self, "_comm_seen"):
            self._comm_seen: set[str] = set()
        if not hasattr(self, "_retention"):
            self._retention = RetentionPlanner(
                self.store, float(os.environ.get("LMX_JOB_RETENTION_DAYS", "7")))
        self._retention.tick()
        if not hasattr(self, "_comm_live_seq"):
            self._comm_live_seq: dict[str, int] = {}
        for m in self.registry.all():
            info = m.info()
            if "kv_usage" in info:
                self.metrics.kv_usage.labels(m.device_id).set(info["kv_usage"])
            if info.get("running"):
                # sampled each maintenance tick: sequences in the engine's batch
                self.metrics.batch_size.labels(m.device_id).observe(info["running"])
            comm = info.get("tp_comm") or {}
            if comm and m.device_id not in self._comm_seen:
                # the TP group's start-up all-reduce probe (parallel/tp_worker.py)
                self._comm_seen.add(m.device_id)
                for path, by_size in comm.items():
                    for us in by_size.values():
                        self.metrics.allreduce.labels(path).observe(us / 1e6)
            live = info.get("tp_comm_live") or {}
            if live.get("seq", 0) > self._comm_live_seq.get(m.device_id, 0):
                # the engine's latest in-service sample (engine._comm_probe)
                self._comm_live_seq[m.device_id] = live["seq"]
                for path, us in (live.get("us") or {}).items():
                    self.metrics.allreduce.labels(path).observe(us / 1e6)
        from ..devices import rocm_enum
        for idx, t in rocm_enum.gpu_telemetry().items():
            dev = rocm_enum.device_id(idx)
            if "hbm_used_bytes" in t:
                self.metrics.hbm_used.labels(dev).set(t["hbm_used_bytes"])
            if "busy_pct" in t:
                self.metrics.gpu_util.labels(dev).set(t["busy_pct"])

    async def start_background(self, app=None):
        disc = env_int("DISCOVERY_INTERVAL", 0)
        self._tasks.append(asyncio.create_task(asyncio.to_thread(self.discovery.run)))
        if disc > 0:
            self._tasks.append(asyncio.create_task(self._every(disc, self.discovery.run,
                                                               "discovery")))
        try:
            lim.apply_device_limits(self.store)
        except Exception:
            log.exception("device limits")
        li = env_int("DEVICE_LIMITS_INTERVAL", 0)
        if li > 0:
            self._tasks.append(asyncio.create_task(
                self._every(li, lambda: lim.apply_device_limits(self.store), "device limits")))
        self._tasks.append(asyncio.create_task(
            self._every(float(os.environ.get("LMX_MAINTENANCE_INTERVAL", "10")),
                        self._maintenance, "maintenance")))

    async def stop_background(self, app=None):
        for t in self._tasks:
            t.cancel()
        self._tasks.clear()
        if self._hub is not None:
            self._hub.close()
            self._hub = None


def create_core_app(state: CoreState, background: bool = True) -> web.Application:
    app = make_app(state)
    if background:
        app.on_startup.append(state.start_background)
        app.on_cleanup.append(state.stop_background)
    return app
