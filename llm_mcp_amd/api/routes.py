"""Control-plane HTTP routes: jobs, workers, devices, discovery, smart LLM
requests, benchmarks, costs, dashboard, debug, feedback, model stats,
knowledge ingest, catalog sync (reference route table:
core/internal/api/server.go:32-62; handlers: core/internal/api/handlers.go).

Response shapes, status codes and error codes follow the reference; the
defects listed in SURVEY §7.6 are fixed (lease tokens, device concurrency on
every claim path, deadlines enforced, cost + circuit on every completion
path, JobsCreated incremented, documented cost field names as aliases)."""
from __future__ import annotations

import asyncio
import json
import os
import re
import time

from aiohttp import ClientSession, ClientTimeout, web

from ..policy import limits as lim
from ..policy.router import QUALITY_TIMEOUTS, RoutingError, parse_payload_model_device
from ..store.base import COST_PERIODS, iso, parse_iso
from ..utils import tracing
from .helpers import read_json, sse_frame, to_int, write_error, write_json

UUID_RE = re.compile(r"^[0-9a-f]{8}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{4}-[0-9a-f]{12}$")
WORKER_PREFIX = "worker-"



def revive_engine_device(store, tags: dict) -> bool:
    """A worker (re-)registering for an engine device brings that device back
    online: it registers only once its engine is up, so after a crash and a
    supervisor restart this is the recovery signal (the device was taken
    offline by the old worker's report or by lease expiry)."""
    dev = str((tags or {}).get("device_id") or "").strip()
    if not dev:
        return False
    d = store.get_device(dev)
    if d is None or d.get("status") == "online":
        return False
    store.set_device_status(dev, "online", {"recovered_at": time.time()})
    return True


def job_json(j: dict) -> dict:
    """models.Job (core/internal/models/types.go:135-149), RFC3339 times,
    omitempty on lease_until / deadline_at / result / error."""
    out = {"id": j["id"], "kind": j["kind"], "payload": j.get("payload") or {},
           "status": j["status"], "attempts": j["attempts"], "max_attempts": j["max_attempts"],
           "priority": j.get("priority", 0), "queued_at": iso(j.get("queued_at")),
           "updated_at": iso(j.get("updated_at"))}
    if j.get("lease_until"):
        out["lease_until"] = iso(j["lease_until"])
    if j.get("deadline_at"):
        out["deadline_at"] = iso(j["deadline_at"])
    if j.get("result") is not None:
        out["result"] = j["result"]
    if j.get("error"):
        out["error"] = j["error"]
    if j.get("attempt_id"):
        out["attempt_id"] = j["attempt_id"]
    if j.get("progress") is not None and j["status"] == "running":
        out["progress"] = j["progress"]
    return out


def _ago(ts: float | None) -> str:
    if not ts:
        return "unknown"
    d = time.time() - ts
    return f"{int(d // 60)}m ago" if d < 3600 else f"{int(d // 3600)}h ago"


def _is_worker(dev_id: str) -> bool:
    return dev_id.startswith(WORKER_PREFIX)


class ControlPlane:
    def __init__(self, state):
        self.st = state

    @property
    def store(self):
        return self.st.store

    async def db(self, fn, *a, **kw):
        if getattr(self.store, "backend", "memory") == "memory":
            return fn(*a, **kw)
        return await asyncio.to_thread(fn, *a, **kw)

    def max_conc(self) -> int:
        return max(1, to_int(os.environ.get("DEVICE_MAX_CONCURRENCY", "1"), 1) or 1)

    # ------------------------------------------------------------ register --
    def register(self, app: web.Application):
        r = app.router
        r.add_route("*", "/v1/jobs", self.jobs)
        r.add_route("*", r"/v1/jobs/{rest:.*}", self.job_by_id)
        r.add_route("*", "/v1/workers/register", self.worker_register)
        r.add_route("*", "/v1/workers/claim", self.worker_claim)
        r.add_route("*", "/v1/workers/complete", self.worker_complete)
        r.add_route("*", "/v1/workers/fail", self.worker_fail)
        r.add_route("*", "/v1/workers/heartbeat", self.worker_heartbeat)
        r.add_route("*", "/v1/devices/offline", self.device_offline)
        r.add_route("*", "/v1/discovery/run", self.discovery_run)
        r.add_route("*", "/v1/discovery/last", self.discovery_last)
        r.add_route("*", "/v1/discovery/local", self.discovery_local)
        r.add_route("*", "/v1/llm/request", self.llm_request)
        r.add_route("*", "/v1/benchmarks/run", self.benchmark_run)
        r.add_route("*", "/v1/benchmarks", self.benchmarks_list)
        r.add_route("*", "/v1/costs/summary", self.costs_summary)
        r.add_route("*", "/v1/costs/balance", self.costs_balance)
        r.add_route("*", "/v1/dashboard", self.dashboard)
        r.add_route("*", "/v1/debug/health", self.debug_health)
        r.add_route("*", "/v1/debug/actions", self.debug_actions)
        r.add_route("*", "/v1/debug/capacity", self.debug_capacity)
        r.add_route("*", "/v1/debug/test", self.debug_test)
        r.add_route("*", "/v1/feedback", self.feedback)
        r.add_route("*", "/v1/knowledge/ingest", self.knowledge_ingest)
        r.add_route("*", "/v1/models/stats", self.models_stats)
        r.add_route("*", "/v1/models/sync", self.models_sync)
        r.add_route("*", "/v1/models", self.models_list)
        r.add_route("GET", "/v1/alerts/snapshot", self.alerts_snapshot)

    async def alerts_snapshot(self, request):
        """Telemetry input (telemetry/alerts.py): counts, GPU devices, failed jobs."""
        from ..telemetry.alerts import snapshot_from_store
        thr = to_int(os.environ.get("ALERT_FAIL_THRESHOLD", "3"), 3)
        temp = float(os.environ.get("LMX_ALERT_TEMP_C", "95"))
        return write_json(200, await self.db(snapshot_from_store, self.store, self.st.circuit,
                                             thr, temp))

    @staticmethod
    def _guard(request, method):
        if request.method != method:
            return write_error(405, "method_not_allowed", "Method not allowed")
        return None

    @staticmethod
    async def _body(request):
        try:
            body = await read_json(request)
        except (ValueError, UnicodeDecodeError):
            return None
        return body if isinstance(body, dict) else None

    # ---------------------------------------------------------------- jobs --
    async def jobs(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        kind = str(body.get("kind") or "").strip()
        if not kind:
            return write_error(400, "kind_required", "Field kind is required")
        payload = body.get("payload")
        if payload is None:
            payload = {}
        if not isinstance(payload, dict):
            return write_error(400, "invalid_payload", "payload must be a JSON object")
        max_attempts = to_int(body.get("max_attempts"), 0) or 3
        deadline = None
        if str(body.get("deadline_at") or "").strip():
            try:
                deadline = parse_iso(body["deadline_at"])
            except ValueError:
                return write_error(400, "invalid_deadline_at",
                                   "Invalid deadline_at (RFC3339 expected)")
        if kind.startswith(("ollama.", "benchmark.ollama.", "engine.", "benchmark.engine.")):
            model, dev = parse_payload_model_device(payload)
            if model and dev:
                ok, why = await self.db(lim.model_allowed, self.store, dev, model)
                if not ok:
                    return write_error(400, "model_not_allowed", "Model not allowed on device: " + why)
        payload = tracing.tag_payload(payload, tracing.client_request_id(request))
        jid = await self.db(self.store.submit_job, kind, payload, to_int(body.get("priority"), 0),
                            str(body.get("source") or ""), max_attempts, deadline)
        self.st.metrics.jobs_created.labels(kind).inc()
        return write_json(202, {"job_id": jid})

    async def job_by_id(self, request):
        rest = request.match_info.get("rest", "")
        if not rest:
            return write_error(404, "not_found", "Resource not found")
        if rest.endswith("/stream"):
            return await self.job_stream(request, rest[: -len("/stream")])
        if rest.endswith("/attempts") and request.method == "GET":
            jid = rest[: -len("/attempts")]
            if not UUID_RE.match(jid):
                return write_error(404, "not_found", "Resource not found")
            return write_json(200, {"items": [dict(a, started_at=iso(a["started_at"]),
                                                   finished_at=iso(a["finished_at"]))
                                              for a in await self.db(self.store.job_attempts, jid)]})
        if (e := self._guard(request, "GET")):
            return e
        if not UUID_RE.match(rest):
            return write_error(404, "not_found", "Resource not found")
        j = await self.db(self.store.get_job, rest)
        if j is None:
            return write_error(404, "not_found", "Resource not found")
        return write_json(200, job_json(j))

    async def job_stream(self, request, jid):
        """SSE: initial status, then every status change until done/error,
        plus ``event: progress`` frames while the job runs (the worker's
        progress reports: tokens generated so far, ttft).  Change notification
        = the store's job version counter (NOTIFY job_update equivalent), with
        a 15 s fallback re-read."""
        if not UUID_RE.match(jid):
            return write_error(404, "not_found", "Resource not found")
        j = await self.db(self.store.get_job, jid)
        if j is None:
            return write_error(404, "not_found", "Resource not found")
        resp = web.StreamResponse(headers={"Content-Type": "text/event-stream",
                                           "Cache-Control": "no-cache",
                                           "Connection": "keep-alive"})
        await resp.prepare(request)
        last = last_prog = None
        ver = self.store.job_version()
        deadline = time.time() + float(os.environ.get("LMX_JOB_STREAM_MAX_S", "3600"))
        try:
            while time.time() < deadline:
                if j is None:
                    await resp.write(sse_frame("error", {"error": "not_found"}))
                    break
                if j["status"] != last:
                    await resp.write(sse_frame("status", job_json(j)))
                    last = j["status"]
                prog = j.get("progress") if j["status"] == "running" else None
                if prog is not None and prog != last_prog:
                    await resp.write(sse_frame("progress", {"id": j["id"], "progress": prog}))
                    last_prog = prog
                if j["status"] in ("done", "error"):
                    break
                ver = await self.st.job_hub().wait(ver, 15.0)
                j = await self.db(self.store.get_job, jid)
        except (ConnectionResetError, ConnectionError):
            pass
        return resp

    # ------------------------------------------------------------- workers --
    async def worker_register(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        w = body.get("worker") or {}
        wid = str(w.get("id") or "").strip() or f"{WORKER_PREFIX}{time.time_ns()}"
        tags = w.get("tags") or {}
        if isinstance(tags, str):
            try:
                tags = json.loads(tags)
            except ValueError:
                tags = {}
        await self.db(self.store.upsert_device, wid, w.get("name", ""), w.get("platform", ""),
                      w.get("arch", ""), w.get("host", ""), tags, "online")
        await self.db(revive_engine_device, self.store, tags)
        return write_json(200, {"worker_id": wid})

    async def worker_claim(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        wid = str(body.get("worker_id") or "").strip()
        if not wid:
            return write_error(400, "worker_id_required", "Field worker_id is required")
        lease = to_int(body.get("lease_seconds"), 0) or 60
        kinds = [k for k in (body.get("kinds") or []) if isinstance(k, str)]
        wait_ms = min(to_int(body.get("wait_ms"), 0) or 0, 30000)
        j = await self._claim(wid, kinds, lease, str(body.get("device_id") or ""), wait_ms)
        if j is None:
            return write_json(200, {})
        return write_json(200, {"job": job_json(j)})

    async def _claim(self, wid, kinds, lease, device, wait_ms):
        """Claim with an optional long-poll (replaces the worker's 1.5 s idle
        poll: the request returns as soon as a job becomes claimable)."""
        t_end = time.time() + wait_ms / 1000.0
        ver = self.store.job_version()
        while True:
            j = await self.db(self.store.claim_job, wid, kinds, lease, device, self.max_conc(), True)
            if j is not None:
                if j.get("queued_at"):
                    self.st.metrics.queue_wait.labels(j["kind"]).observe(
                        max(0.0, time.time() - j["queued_at"]))
                return j
            left = t_end - time.time()
            if left <= 0:
                return None
            ver = await self.st.job_hub().wait(ver, min(left, 5.0))

    def _record_cost(self, jid, metrics: dict):
        """RecordCost (handlers.go:836-869): llm_costs row from worker metrics."""
        tin, tout = to_int(metrics.get("tokens_in"), 0), to_int(metrics.get("tokens_out"), 0)
        prov, model = metrics.get("provider") or "", metrics.get("model") or ""
        if (tin == 0 and tout == 0) or not prov or not model:
            return
        cost = self.store.calculate_job_cost(model, tin, tout)
        self.store.insert_cost(jid, model, prov, tin, tout, cost)
        self.st.metrics.chat_cost.labels(model, prov).inc(cost)

    async def worker_complete(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        wid, jid = str(body.get("worker_id") or "").strip(), str(body.get("job_id") or "").strip()
        if not wid or not jid:
            return write_error(400, "worker_id_job_id_required",
                               "Fields worker_id and job_id are required")
        result = body.get("result") or {}
        metrics = body.get("metrics") or {}
        ok = await self.db(self.store.complete_job, jid, wid, result, metrics,
                           str(body.get("attempt_id") or body.get("lease_token") or ""))
        if not ok:
            return write_error(409, "lease_lost", "Job is not leased by this worker")
        await self.db(self._record_cost, jid, metrics if isinstance(metrics, dict) else {})
        dev = (result.get("device_id") if isinstance(result, dict) else None) or \
            ((await self.db(self.store.get_job, jid)) or {}).get("device_id")
        if dev:
            self.st.circuit.record(dev, True)
        return write_json(200, {"ok": True})

    async def worker_fail(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        wid, jid = str(body.get("worker_id") or "").strip(), str(body.get("job_id") or "").strip()
        if not wid or not jid:
            return write_error(400, "worker_id_job_id_required",
                               "Fields worker_id and job_id are required")
        j = await self.db(self.store.get_job, jid)
        if j is None:
            return write_error(404, "not_found", "Resource not found")
        st = await self.db(self.store.fail_job, jid, wid, str(body.get("error") or ""),
                           body.get("metrics") or {},
                           str(body.get("attempt_id") or body.get("lease_token") or ""))
        if st is None:
            return write_error(409, "lease_lost", "Job is not leased by this worker")
        dev = j.get("device_id") or (j.get("payload") or {}).get("device_id")
        if dev:
            self.st.circuit.record(dev, False)
        return write_json(200, {"ok": True, "status": st})

    async def worker_heartbeat(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        wid, jid = str(body.get("worker_id") or "").strip(), str(body.get("job_id") or "").strip()
        if not wid or not jid:
            return write_error(400, "worker_id_job_id_required",
                               "Fields worker_id and job_id are required")
        ext = to_int(body.get("extend_seconds"), 0) or 30
        prog = body.get("progress")
        ok = await self.db(self.store.heartbeat, jid, wid, ext,
                           str(body.get("attempt_id") or body.get("lease_token") or ""),
                           prog if isinstance(prog, dict) else None)
        await self.db(self.store.set_device_status, wid, "online")
        return write_json(200, {"ok": bool(ok)})

    async def device_offline(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        dev = str(body.get("device_id") or "").strip()
        if not dev:
            return write_error(400, "device_id_required", "Field device_id is required")
        await self.db(self.store.set_device_status, dev, "offline",
                      {"last_error": body.get("reason", ""), "last_error_at": iso(time.time())})
        n = await self.db(self.store.release_device_leases, dev)
        # every job still leased on the device failed there: feed the breaker
        # once per released lease (at least once for the report itself) -- the
        # workers' own fail reports for those jobs race this release and may
        # come back lease_lost, so they cannot be relied on to trip it
        for _ in range(max(1, int(n or 0))):
            self.st.circuit.record(dev, False)
        return write_json(200, {"ok": True, "released": int(n or 0)})

    # ----------------------------------------------------------- discovery --
    async def discovery_run(self, request):
        if (e := self._guard(request, "POST")):
            return e
        try:
            await asyncio.wait_for(asyncio.to_thread(self.st.discovery.run), 15)
        except Exception:
            return write_error(500, "discovery_failed", "Discovery run failed")
        return write_json(200, {"status": "ok"})

    async def discovery_last(self, request):
        if (e := self._guard(request, "GET")):
            return e
        return write_json(200, {"last_run": iso(self.st.discovery.last_run()) or ""})

    async def discovery_local(self, request):
        """This node's devices (polled by peers: the Tailscale-scan replacement)."""
        devs = [{k: v for k, v in d.items() if k != "models"}
                for d in await asyncio.to_thread(self.st.discovery.local_devices)]
        return write_json(200, {"devices": devs})

    # ---------------------------------------------------------------- llm ---
    async def llm_request(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        try:
            provider, kind, payload = await self.db(self.st.router.route_llm, body)
        except RoutingError as ex:
            return write_error(400, "routing_failed", str(ex))
        deadline = None
        if str(body.get("deadline_at") or "").strip():
            try:
                deadline = parse_iso(body["deadline_at"])
            except ValueError:
                return write_error(400, "invalid_deadline_at",
                                   "Invalid deadline_at (RFC3339 expected)")
        if deadline is None:
            secs = QUALITY_TIMEOUTS.get(str(body.get("quality") or "").strip().lower())
            if secs:
                deadline = time.time() + secs
        if isinstance(payload, dict):
            payload = tracing.tag_payload(payload, tracing.client_request_id(request))
        jid = await self.db(self.store.submit_job, kind, payload, to_int(body.get("priority"), 0),
                            str(body.get("source") or ""), to_int(body.get("max_attempts"), 0) or 3,
                            deadline)
        self.st.metrics.jobs_created.labels(kind).inc()
        return write_json(202, {"job_id": jid, "provider": provider, "kind": kind})

    # ---------------------------------------------------------- benchmarks --
    async def benchmark_run(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        provider = str(body.get("provider") or "local").strip().lower()
        task = str(body.get("task_type") or "generate").strip().lower()
        if provider not in ("local", "ollama", "engine"):
            return write_error(400, "provider_not_supported",
                               "Benchmarks run on local GPU engines only")
        kind = ("benchmark.ollama." if provider == "ollama" else "benchmark.engine.") + task
        runs = to_int(body.get("runs"), 0) or 1
        prio = to_int(body.get("priority"), 0) or 1
        payload = {"model": body.get("model", ""), "prompt": body.get("prompt", "")}
        for k in ("max_tokens", "prompt_tokens", "concurrency"):
            if body.get(k) is not None:
                payload[k] = body[k]
        dev = str(body.get("device_id") or "").strip()
        if dev:
            if body.get("model"):
                ok, why = await self.db(lim.model_allowed, self.store, dev, body["model"])
                if not ok:
                    return write_error(400, "model_not_allowed",
                                       "Model not allowed on device: " + why)
            d = await self.db(self.store.get_device, dev)
            if d is None:
                return write_error(400, "device_not_found", "Device not found")
            payload["device_id"] = dev
        ids = []
        for _ in range(runs):
            ids.append(await self.db(self.store.submit_job, kind, payload, prio, "benchmark", 2))
            self.st.metrics.jobs_created.labels(kind).inc()
        return write_json(202, {"job_ids": ids, "kind": kind})

    async def benchmarks_list(self, request):
        if (e := self._guard(request, "GET")):
            return e
        n = to_int(request.query.get("limit"), 20) or 20
        if n <= 0 or n > 200:
            n = 20
        items = [{"device_id": b["device_id"], "model_id": b["model_id"],
                  "task_type": b["task_type"], "tokens_in": b["tokens_in"],
                  "tokens_out": b["tokens_out"], "latency_ms": b["latency_ms"], "tps": b["tps"],
                  "created_at": iso(b["created_at"]), "meta": b.get("meta") or {}}
                 for b in await self.db(self.store.list_benchmarks, n)]
        return write_json(200, {"items": items})

    # --------------------------------------------------------------- costs --
    async def costs_summary(self, request):
        if (e := self._guard(request, "GET")):
            return e
        period = request.query.get("period") or "day"
        if period not in COST_PERIODS:
            return write_error(400, "invalid_period", "Invalid period: day, week, month")
        s = await self.db(self.store.cost_summary, time.time() - COST_PERIODS[period])
        out = {"period": period, "total_cost": s["total_cost"], "total_jobs": s["total_jobs"],
               "by_provider": s["by_provider"],
               # documented field names (doc/README.md:169-177) as aliases
               "total_cost_usd": s["total_cost"], "requests": s["total_jobs"]}
        return write_json(200, out)

    async def costs_balance(self, request):
        if (e := self._guard(request, "GET")):
            return e
        res = {"openrouter_balance_usd": None, "spend_today_usd": 0, "spend_week_usd": 0,
               "spend_month_usd": 0, "top_models": []}
        key = os.environ.get("OPENROUTER_API_KEY", "")
        if key and key != "not-used" and os.environ.get("LMX_ALLOW_CLOUD", "0") == "1":
            try:
                async with ClientSession(timeout=ClientTimeout(total=10)) as s:
                    async with s.get(os.environ.get("OPENROUTER_BASE_URL",
                                                    "https://openrouter.ai/api/v1") + "/auth/key",
                                     headers={"Authorization": "Bearer " + key}) as r:
                        d = (await r.json()).get("data", {})
                left = d.get("limit_remaining")
                bal = left if left is not None else (
                    (d["limit"] - d.get("usage", 0)) if d.get("limit") is not None else 0.0)
                res["openrouter_balance_usd"] = bal
                res["openrouter_usage_usd"] = d.get("usage", 0)
                self.st.metrics.openrouter_balance.set(bal)
            except Exception:
                pass
        now = time.time()
        for k, per in (("spend_today_usd", "day"), ("spend_week_usd", "week"),
                       ("spend_month_usd", "month")):
            res[k] = (await self.db(self.store.cost_summary, now - COST_PERIODS[per]))["total_cost"]
        res["top_models"] = await self.db(self.store.cost_top_models, now - COST_PERIODS["month"])
        return write_json(200, res)

    # ----------------------------------------------------------- dashboard --
    def _engine_devices(self) -> list[dict]:
        out = []
        running = {}
        for j in self.store.running_jobs(100000):
            d = j.get("device_id") or (j.get("payload") or {}).get("device_id")
            if d:
                running[d] = running.get(d, 0) + 1
        dms = self.store.list_device_models(available_only=True)
        for d in self.store.list_devices():
            tags = d.get("tags") or {}
            if _is_worker(d["id"]) or not (tags.get("engine") or tags.get("ollama")):
                continue
            names = sorted(dm["model_id"] for dm in dms if dm["device_id"] == d["id"])
            out.append({"id": d["id"], "name": d.get("name") or d["id"],
                        "status": d.get("status", "unknown"), "platform": d.get("platform", ""),
                        "arch": d.get("arch", ""), "host": d.get("host", ""),
                        "models_count": len(names), "model_names": names,
                        "running_jobs": running.get(d["id"], 0),
                        "latency_ms": tags.get("latency_ms"),
                        "last_seen": iso(d.get("last_seen")), "_last_seen": d.get("last_seen"),
                        "tags": tags, "stats": self.store.device_stats_7d(d["id"]),
                        "circuit": self.st.circuit.status(d["id"]),
                        "circuit_trips": self.st.circuit.trips.get(d["id"], 0)})
        out.sort(key=lambda x: (x["status"] != "online", x["name"]))
        return out

    def _capacity_of(self, dev: dict) -> int:
        cap = (dev.get("tags") or {}).get("capacity")
        if not cap:
            lim_ = self.store.get_device_limits(dev["id"]) or {}
            cap = lim_.get("max_concurrency")
        return int(cap or self.max_conc())

    def _hosts(self, devices: list[dict]) -> list[dict]:
        """Host -> Node hierarchy: host = machine, node = GPU (or TP group)."""
        hosts: dict[str, dict] = {}
        for d in devices:
            hid = d.get("host") or d["id"].split(":")[0]
            h = hosts.setdefault(hid, {"id": hid, "name": hid, "platform": d["platform"],
                                       "status": "offline", "orchestration": "native",
                                       "last_seen": None, "_ls": 0, "nodes": [],
                                       "total_models": 0, "total_running": 0, "total_slots": 0,
                                       "stats": None, "circuit": "ok"})
            if d["status"] == "online":
                h["status"] = "online"
            if (d.get("_last_seen") or 0) > h["_ls"]:
                h["_ls"] = d["_last_seen"]
                h["last_seen"] = d["last_seen"]
            names = d["model_names"]
            emb = any("embed" in n for n in names)
            chat = any("embed" not in n for n in names)
            role = "mixed" if emb and chat else ("embed" if emb else "chat")
            tags = d.get("tags") or {}
            h["nodes"].append({"gpu": tags.get("gpu_index"), "device_id": d["id"], "role": role,
                               "models_count": d["models_count"], "model_names": names,
                               "latency_ms": d.get("latency_ms"), "running_jobs": d["running_jobs"],
                               "stats": d["stats"], "circuit": d["circuit"],
                               "hbm_gb": tags.get("hbm_gb"), "gfx": tags.get("gfx")})
            h["total_models"] += d["models_count"]
            h["total_running"] += d["running_jobs"]
            h["total_slots"] += self._capacity_of(d)
            if d["circuit"] == "degraded" or (d["circuit"] == "probe" and h["circuit"] == "ok"):
                h["circuit"] = d["circuit"]
        for h in hosts.values():
            tot = sum(n["stats"]["total_jobs_7d"] for n in h["nodes"] if n["stats"])
            done = sum(n["stats"]["done_jobs_7d"] for n in h["nodes"] if n["stats"])
            if tot:
                lat = [n["stats"]["avg_latency_ms"] * n["stats"]["total_jobs_7d"]
                       for n in h["nodes"] if n["stats"] and n["stats"]["avg_latency_ms"]]
                h["stats"] = {"total_jobs_7d": tot, "done_jobs_7d": done,
                              "success_rate": done * 100.0 / tot,
                              "avg_latency_ms": int(sum(lat) / tot) if lat else 0}
            del h["_ls"]
        return sorted(hosts.values(), key=lambda h: (h["status"] != "online", h["name"]))

    def _workers_online(self) -> int:
        now = time.time()
        return sum(1 for d in self.store.list_devices() if _is_worker(d["id"]) and
                   d.get("status") == "online" and (d.get("last_seen") or 0) > now - 600)

    @staticmethod
    def _issues(hosts, jobs, workers_online) -> list[str]:
        issues = []
        for h in hosts:
            if h["status"] != "online" and h["last_seen"]:
                issues.append(f"Host '{h['name']}' offline (last seen "
                              f"{_ago(parse_iso(h['last_seen']))})")
        for h in hosts:
            if h["circuit"] == "degraded":
                issues.append(f"Host '{h['name']}' circuit degraded")
        for h in hosts:
            s = h.get("stats")
            if s and s["total_jobs_7d"] >= 5 and s["success_rate"] < 80:
                issues.append(f"Host '{h['name']}' low success rate: {s['success_rate']:.1f}%")
        q, r = jobs.get("queued", 0), jobs.get("running", 0)
        if q > 0 and r == 0 and workers_online > 0:
            issues.append(f"Queue stuck: {q} jobs queued but no workers processing")
        if q > 10:
            issues.append(f"Queue backlog: {q} jobs waiting")
        return issues

    def _dashboard(self) -> dict:
        st = self.store
        jobs = {k: v for k, v in st.job_counts().items() if v}
        bench: dict[str, int] = {}
        if hasattr(st, "kind_counts"):     # counted natively: O(jobs) in C++, no row copies
            bench = {k: v for k, v in st.kind_counts("benchmark.").items() if v}
        else:
            for s_ in ("queued", "running", "done", "error"):
                for j in st.list_jobs(s_, 0) if hasattr(st, "list_jobs") else []:
                    if j["kind"].startswith("benchmark."):
                        bench[s_] = bench.get(s_, 0) + 1
        running = []
        for j in st.running_jobs(10):
            p = j.get("payload") or {}
            running.append({"id": j["id"], "kind": j["kind"], "model": p.get("model", ""),
                            "provider": p.get("provider", ""),
                            "device_id": j.get("device_id") or p.get("device_id", ""),
                            "updated_at": iso(j.get("updated_at"))})
        devices = self._engine_devices()
        hosts = self._hosts(devices)
        wo = self._workers_online()
        now = time.time()
        costs = {k: st.cost_summary(now - COST_PERIODS[p])["total_cost"]
                 for k, p in (("today", "day"), ("week", "week"), ("month", "month"))}
        models = {dm["model_id"] for dm in st.list_device_models(available_only=True)}
        for d in devices:
            d.pop("_last_seen", None)
        out = {"jobs": jobs, "benchmarks": bench, "running_jobs": running, "devices": devices,
               "hosts": hosts, "workers_online": wo, "issues": self._issues(hosts, jobs, wo),
               "costs": costs, "models_count": len(models), "updated_at": iso(now)}
        eng = getattr(self.st, "registry", None)
        if eng is not None:
            out["engines"] = [m.info() for m in eng.all()]
        return out

    async def dashboard(self, request):
        if (e := self._guard(request, "GET")):
            return e
        return write_json(200, await self.db(self._dashboard))

    # --------------------------------------------------------------- debug --
    def _debug_health(self) -> dict:
        st = self.store
        worst = ["ok"]

        def set_worst(s):
            if s == "error" or (s == "warning" and worst[0] != "error"):
                worst[0] = s

        t0 = time.time()
        db = {"status": "ok", "backend": getattr(st, "backend", "?")}
        try:
            st.ping()
            db["latency_ms"] = int((time.time() - t0) * 1000)
        except Exception as ex:
            db.update(status="error", error=str(ex))
            set_worst("error")
        counts = st.job_counts()
        stuck = st.stuck_jobs()
        queue = {"status": "ok", "queued": counts.get("queued", 0),
                 "running": counts.get("running", 0), "stuck": stuck}
        qd = [j["queued_at"] for j in (st.list_jobs("queued", 0) if hasattr(st, "list_jobs")
                                       else []) if j.get("queued_at")]
        if qd:
            queue["oldest_queued_sec"] = int(time.time() - min(qd))
        if stuck:
            queue["status"] = "warning"
            set_worst("warning")
        devs = [d for d in st.list_devices() if not _is_worker(d["id"]) and
                ((d.get("tags") or {}).get("engine") or (d.get("tags") or {}).get("ollama"))]
        on = sum(1 for d in devs if d.get("status") == "online")
        hosts = {"status": "ok", "total": len(devs), "online": on, "offline": len(devs) - on}
        if len(devs) - on > 0:
            hosts["status"] = "warning"
            set_worst("warning")
        if on == 0 and devs:
            hosts["status"] = "error"
            set_worst("error")
        wo = self._workers_online()
        workers = {"status": "ok", "online": wo, "capacity": wo * self.max_conc()}
        if wo == 0:
            workers["status"] = "warning"
            set_worst("warning")
        engines = {"status": "ok", "count": 0}
        reg = getattr(self.st, "registry", None)
        if reg is not None:
            engines["count"] = len(reg.all())
            engines["models"] = reg.model_ids()
        issues = [f"Host '{d.get('name') or d['id']}' offline (last seen "
                  f"{_ago(d.get('last_seen'))})" for d in devs if d.get("status") != "online"]
        if stuck:
            issues.append(f"{stuck} jobs with expired lease")
        if queue["queued"] > 0 and queue["running"] == 0 and wo > 0:
            issues.append(f"Queue stuck: {queue['queued']} jobs queued but no workers processing")
        if queue["queued"] > 10:
            issues.append(f"Queue backlog: {queue['queued']} jobs waiting")
        return {"status": worst[0], "version": self.st.version,
                "checks": {"database": db, "queue": queue, "hosts": hosts, "workers": workers,
                           "engines": engines}, "issues": issues}

    async def debug_health(self, request):
        if (e := self._guard(request, "GET")):
            return e
        return write_json(200, await self.db(self._debug_health))

    ACTIONS = [
        ("GET", "/health", "Service health", "curl http://localhost:8080/health"),
        ("GET", "/version", "Service version", "curl http://localhost:8080/version"),
        ("GET", "/v1/dashboard", "Full snapshot: jobs, hosts/GPUs, engines, costs, issues",
         "curl http://localhost:8080/v1/dashboard | jq ."),
        ("POST", "/v1/jobs", "Create a queued job",
         "curl -X POST http://localhost:8080/v1/jobs -d '{\"kind\":\"engine.generate\","
         "\"payload\":{\"model\":\"llama-3-8b\",\"prompt\":\"Hello\"}}'"),
        ("GET", "/v1/jobs/{id}", "Job status (payload, result, attempts)",
         "curl http://localhost:8080/v1/jobs/<id>"),
        ("GET", "/v1/jobs/{id}/stream", "SSE job status updates",
         "curl -N http://localhost:8080/v1/jobs/<id>/stream"),
        ("POST", "/v1/llm/request", "Routed LLM request (classic or quality-based smart routing)",
         "curl -X POST http://localhost:8080/v1/llm/request -d '{\"task\":\"chat\","
         "\"quality\":\"standard\",\"prompt\":\"Hello\"}'"),
        ("POST", "/v1/workers/register", "Register a worker",
         "curl -X POST http://localhost:8080/v1/workers/register -d '{\"worker\":{\"id\":\"w1\"}}'"),
        ("POST", "/v1/workers/claim", "Claim a job (lease; optional wait_ms long-poll)",
         "curl -X POST http://localhost:8080/v1/workers/claim -d '{\"worker_id\":\"w1\"}'"),
        ("POST", "/v1/workers/complete", "Complete a job (attempt_id = lease token)",
         "curl -X POST http://localhost:8080/v1/workers/complete -d '{\"worker_id\":\"w1\","
         "\"job_id\":\"<id>\",\"attempt_id\":\"<token>\",\"result\":{}}'"),
        ("POST", "/v1/workers/fail", "Fail a job (requeued until max_attempts)",
         "curl -X POST http://localhost:8080/v1/workers/fail -d '{\"worker_id\":\"w1\","
         "\"job_id\":\"<id>\",\"error\":\"timeout\"}'"),
        ("POST", "/v1/workers/heartbeat", "Extend a job lease",
         "curl -X POST http://localhost:8080/v1/workers/heartbeat -d '{\"worker_id\":\"w1\","
         "\"job_id\":\"<id>\",\"extend_seconds\":30}'"),
        ("POST", "/v1/devices/offline", "Mark a device offline (its leases are released)",
         "curl -X POST http://localhost:8080/v1/devices/offline -d '{\"device_id\":\"node:gpu0\"}'"),
        ("POST", "/v1/discovery/run", "Re-enumerate GPUs / peer nodes",
         "curl -X POST http://localhost:8080/v1/discovery/run"),
        ("GET", "/v1/discovery/last", "Last discovery run", "curl http://localhost:8080/v1/discovery/last"),
        ("POST", "/v1/benchmarks/run", "Queue GPU benchmark jobs",
         "curl -X POST http://localhost:8080/v1/benchmarks/run -d '{\"model\":\"llama-3-8b\","
         "\"runs\":3}'"),
        ("GET", "/v1/benchmarks", "Recent benchmarks", "curl 'http://localhost:8080/v1/benchmarks?limit=10'"),
        ("GET", "/v1/costs/summary", "Spend per provider", "curl 'http://localhost:8080/v1/costs/summary?period=week'"),
        ("GET", "/v1/costs/balance", "Spend windows + top models", "curl http://localhost:8080/v1/costs/balance"),
        ("GET", "/v1/debug/health", "Deep health check", "curl http://localhost:8080/v1/debug/health"),
        ("GET", "/v1/debug/actions", "This catalogue", "curl http://localhost:8080/v1/debug/actions"),
        ("GET", "/v1/debug/capacity", "Slots / utilisation per host and GPU",
         "curl http://localhost:8080/v1/debug/capacity"),
        ("POST", "/v1/debug/test", "Smoke test: store, engines, job pipeline",
         "curl -X POST http://localhost:8080/v1/debug/test"),
        ("POST", "/v1/chat/completions", "OpenAI chat completions (sync / SSE) on local GPUs",
         "curl -N http://localhost:8080/v1/chat/completions -d '{\"model\":\"llama-3-8b\","
         "\"stream\":true,\"messages\":[{\"role\":\"user\",\"content\":\"hi\"}]}'"),
        ("POST", "/v1/embeddings", "OpenAI embeddings on local GPUs",
         "curl -X POST http://localhost:8080/v1/embeddings -d '{\"model\":\"nomic-embed-text\","
         "\"input\":\"Hello world\"}'"),
        ("GET", "/v1/models", "Served models", "curl http://localhost:8080/v1/models"),
        ("GET", "/metrics", "Prometheus metrics", "curl http://localhost:8080/metrics"),
    ]

    async def debug_actions(self, request):
        if (e := self._guard(request, "GET")):
            return e
        eps = [{"method": m, "path": p, "description": d, "example": x}
               for m, p, d, x in self.ACTIONS]
        return write_json(200, {"endpoints": eps, "total": len(eps)})

    def _capacity(self) -> dict:
        devices = self._engine_devices()
        hosts = self._hosts(devices)
        caps, tot, used = [], 0, 0
        for h in hosts:
            slots, u = h["total_slots"], h["total_running"]
            tot += slots
            used += u
            caps.append({"name": h["name"], "status": h["status"], "slots": slots, "used": u,
                         "free": max(0, slots - u),
                         "utilization_pct": (u * 100.0 / slots) if slots else 0.0,
                         "models": h["total_models"], "circuit": h["circuit"],
                         "gpus": [{"device_id": n["device_id"], "running": n["running_jobs"],
                                   "hbm_gb": n["hbm_gb"]} for n in h["nodes"]]})
        wo = self._workers_online()
        out = {"total_slots": tot, "used_slots": used, "free_slots": max(0, tot - used),
               "utilization_pct": (used * 100.0 / tot) if tot else 0.0, "hosts": caps,
               "workers": {"online": wo, "total_capacity": wo * self.max_conc()}}
        reg = getattr(self.st, "registry", None)
        if reg is not None:
            out["engines"] = [m.info() for m in reg.all()]
        return out

    async def debug_capacity(self, request):
        if (e := self._guard(request, "GET")):
            return e
        return write_json(200, await self.db(self._capacity))

    async def debug_test(self, request):
        if (e := self._guard(request, "POST")):
            return e
        start = time.time()
        status, results, issues = "pass", [], []
        t0 = time.time()
        try:
            await self.db(self.store.ping)
            results.append({"name": "db_ping", "status": "pass",
                            "ms": int((time.time() - t0) * 1000),
                            "detail": f"store ({self.store.backend}) reachable"})
        except Exception as ex:
            results.append({"name": "db_ping", "status": "fail",
                            "ms": int((time.time() - t0) * 1000), "detail": f"Error: {ex}"})
            status = "fail"
            issues.append("Database unreachable")
        t0 = time.time()
        devs = await self.db(self.store.list_devices)
        dms = await self.db(self.store.list_device_models, None, True)
        results.append({"name": "db_read", "status": "pass", "ms": int((time.time() - t0) * 1000),
                        "detail": f"Read {len(devs)} devices, {len(dms)} models"})
        # engine_ping: one tiny generation per local chat engine (GPU health probe)
        t0 = time.time()
        reg = getattr(self.st, "registry", None)
        engines = [m for m in (reg.all() if reg else []) if m.kind == "chat"]
        ok = 0
        for m in engines:
            try:
                from ..engine.engine import SamplingParams
                toks, _, fin = await asyncio.wait_for(m.engine.complete(
                    m.tokenizer.encode("ping"), SamplingParams(max_tokens=1, temperature=0)), 10)
                if toks:
                    ok += 1
                    self.st.circuit.record(m.device_id, True)
                else:
                    issues.append(f"Engine '{m.model_id}' on {m.device_id} returned no token")
            except Exception as ex:
                issues.append(f"Engine '{m.model_id}' on {m.device_id} failed: {ex}")
                self.st.circuit.record(m.device_id, False)
        est = "pass" if ok == len(engines) else "warn"
        if est == "warn" and status == "pass":
            status = "warn"
        results.append({"name": "engine_ping", "status": est, "ms": int((time.time() - t0) * 1000),
                        "detail": f"{ok}/{len(engines)} engines reachable"})
        t0 = time.time()
        try:
            jid = await self.db(self.store.submit_job, "debug.test", {"smoke_test": True}, -1,
                                "debug", 1, None, "done")
            results.append({"name": "job_create", "status": "pass",
                            "ms": int((time.time() - t0) * 1000),
                            "detail": f"Job {jid[:8]} created and cleaned"})
        except Exception as ex:
            results.append({"name": "job_create", "status": "fail",
                            "ms": int((time.time() - t0) * 1000), "detail": f"Error: {ex}"})
            status = "fail"
            issues.append("Cannot create jobs in the store")
        return write_json(200, {"status": status, "duration_ms": int((time.time() - start) * 1000),
                                "results": results, "issues": issues})

    # ----------------------------------------------------- feedback / stats --
    async def feedback(self, request):
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        model = str(body.get("model") or "")
        if not model:
            return write_error(400, "model_required", "Field 'model' is required")
        rating = body.get("rating")
        if rating not in ("good", "bad"):
            return write_error(400, "invalid_rating", "Rating must be 'good' or 'bad'")
        await self.db(self.store.feedback, model, rating == "good")
        return write_json(200, {"status": "ok", "model": model, "rating": rating})

    def _model_stats(self) -> list[dict]:
        ranks = {r["model_id"]: r for r in self.store.list_model_rankings()}
        stats = {s["model_id"]: s for s in self.store.model_stats()}
        ids = set(ranks) | set(stats)
        out = []
        for mid in ids:
            r, s = ranks.get(mid, {}), stats.get(mid, {})
            pos, neg = s.get("feedback_positive", 0), s.get("feedback_negative", 0)
            m = self.store.get_model(mid) or {}
            out.append({
                "model_id": mid, "display_name": r.get("display_name", mid),
                "provider": r.get("provider", m.get("provider", "local")),
                "category_scores": r.get("category_scores", {}),
                "price_in_1m": r.get("price_in_1m", 0.0), "price_out_1m": r.get("price_out_1m", 0.0),
                "context_k": r.get("context_k", m.get("context_k")),
                "total_requests": s.get("total_requests", 0),
                "total_tokens_in": s.get("total_tokens_in", 0),
                "total_tokens_out": s.get("total_tokens_out", 0),
                "total_cost_usd": s.get("total_cost_usd", 0.0),
                "avg_duration_ms": int(s.get("avg_duration_ms", 0)),
                "error_count": s.get("error_count", 0), "success_rate": s.get("success_rate", 0.0),
                "feedback_score": (pos * 100.0 / (pos + neg)) if pos + neg else 0.0,
                "last_used_at": iso(s.get("last_used_at"))})
        out.sort(key=lambda x: -x["total_cost_usd"])
        return out

    async def models_stats(self, request):
        if (e := self._guard(request, "GET")):
            return e
        ms = await self.db(self._model_stats)
        return write_json(200, {"models": ms, "count": len(ms)})

    async def models_list(self, request):
        """OpenAI-style model list of the locally served models."""
        reg = getattr(self.st, "registry", None)
        data = [{"id": mid, "object": "model", "owned_by": "local", "created": 0}
                for mid in (reg.model_ids() if reg else [])]
        return write_json(200, {"object": "list", "data": data})

    # ------------------------------------------------------ external proxies --
    async def knowledge_ingest(self, request):
        """Pass-through to LightRAG / mem0 (no default API key is baked in:
        LIGHTRAG_API_KEY must be configured -- fixes the reference's hard-coded
        key, handlers.go:2895)."""
        if (e := self._guard(request, "POST")):
            return e
        body = await self._body(request)
        if body is None:
            return write_error(400, "invalid_json", "Invalid JSON body")
        text = str(body.get("text") or "")
        target = body.get("target") or "lightrag"
        meta = body.get("metadata") or {}
        if target == "lightrag":
            if len(text) < 100:
                return write_error(400, "text_too_short",
                                   "Text must be at least 100 characters for LightRAG")
            head = f"# Source-Type: {meta.get('source_type', 'agent-learning')}\n"
            if meta.get("domain"):
                head += f"# Domain: {meta['domain']}\n"
            head += f"# Ingested: {time.strftime('%Y-%m-%d')}\n\n"
            url = os.environ.get("LIGHTRAG_URL", "http://lightrag:9621") + "/documents/text"
            hdr = {"X-API-Key": os.environ["LIGHTRAG_API_KEY"]} \
                if os.environ.get("LIGHTRAG_API_KEY") else {}
            payload = {"text": head + text, "description": meta.get("topic", "")}
            timeout, err = 30, "lightrag_error"
        elif target == "mem0":
            if len(text) < 10:
                return write_error(400, "text_too_short",
                                   "Text must be at least 10 characters for mem0")
            url = os.environ.get("MEM0_URL", "http://mem0:8800") + "/v1/memories/"
            hdr = {}
            payload = {"messages": [{"role": "user", "content": text}],
                       "user_id": body.get("user_id") or "default"}
            timeout, err = 15, "mem0_error"
        else:
            return write_error(400, "invalid_target", "Target must be 'lightrag' or 'mem0'")
        try:
            async with ClientSession(timeout=ClientTimeout(total=timeout)) as s:
                async with s.post(url, json=payload, headers=hdr) as r:
                    data = await r.read()
                    return web.Response(status=r.status, body=data,
                                        content_type="application/json")
        except Exception as ex:
            return write_error(502, err, str(ex))

    async def models_sync(self, request):
        """Catalog sync of OpenRouter rankings (cloud; only with LMX_ALLOW_CLOUD=1).
        Local models are synced by discovery from the engines themselves."""
        if (e := self._guard(request, "POST")):
            return e
        if os.environ.get("LMX_ALLOW_CLOUD", "0") != "1":
            # local catalogue refresh instead
            await asyncio.to_thread(self.st.discovery.run)
            return write_json(200, {"status": "ok", "synced": len(self.store.list_models()),
                                    "categories": [], "source": "local"})
        from ..planner.catalog import sync_openrouter
        try:
            res = await sync_openrouter(self.store)
        except Exception as ex:
            return write_error(502, "sync_failed", str(ex))
        return write_json(200, res)
