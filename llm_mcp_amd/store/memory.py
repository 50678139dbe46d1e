"""In-process store: the job queue is the native C++ lease queue
(csrc/runtime/job_queue.cpp, optional crash-durable journal), the catalog
tables (devices, models, device_models, benchmarks, device_limits, llm_costs,
model_rankings, model_stats, device_metrics, pricing) live in process memory
behind one lock, optionally snapshotted to a JSON file.

Semantics mirror the reference SQL (db/init/01_core.sql, db/migrations/*,
core/internal/api/handlers.go); SURVEY §7.6 defects are fixed (see
job_queue.h)."""
from __future__ import annotations

import json
import os
import threading
import time
import uuid

from ..native import runtime
from .base import now


def _ms(t: float | None) -> int:
    return 0 if t is None else int(t * 1000)


def _s(ms: int) -> float | None:
    return None if not ms else ms / 1000.0


def _loads(s: str, default):
    if not s:
        return default
    try:
        return json.loads(s)
    except ValueError:
        return default


class MemoryStore:
    backend = "memory"

    def __init__(self, journal_path: str = "", snapshot_path: str = "", clock=None):
        rt = runtime()
        self.q = rt.JobQueue(journal_path)
        self.clock = clock or now
        self.snapshot_path = snapshot_path
        self._lock = threading.RLock()
        self.devices: dict[str, dict] = {}
        self.models: dict[str, dict] = {}
        self.pricing: dict[str, tuple[float, float]] = {}
        self.device_models: dict[tuple[str, str], dict] = {}
        self.benchmarks: list[dict] = []
        self.device_limits: dict[str, dict] = {}
        self.costs: list[dict] = []
        self.rankings: dict[str, dict] = {}
        self.stats: dict[str, dict] = {}
        self.device_metrics: list[dict] = []
        self.progress: dict[str, dict] = {}  # running job -> last worker progress report
        if snapshot_path and os.path.exists(snapshot_path):
            self._load_snapshot()

    # ------------------------------------------------------------ snapshot --
    _TABLES = ("devices", "models", "benchmarks", "device_limits", "costs", "rankings", "stats")

    def save_snapshot(self) -> None:
        if not self.snapshot_path:
            return
        with self._lock:
            data = {t: getattr(self, t) for t in self._TABLES}
            data["pricing"] = {k: list(v) for k, v in self.pricing.items()}
            data["device_models"] = [dict(v) for v in self.device_models.values()]
        tmp = self.snapshot_path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(data, f)
        os.replace(tmp, self.snapshot_path)

    def _load_snapshot(self) -> None:
        with open(self.snapshot_path) as f:
            data = json.load(f)
        for t in self._TABLES:
            if t in data:
                setattr(self, t, data[t])
        self.pricing = {k: tuple(v) for k, v in data.get("pricing", {}).items()}
        self.device_models = {(d["device_id"], d["model_id"]): d
                              for d in data.get("device_models", [])}

    def ping(self) -> bool:
        return True

    # ---------------------------------------------------------------- jobs --
    def _job(self, r: dict) -> dict:
        return {"id": r["id"], "kind": r["kind"], "payload": _loads(r["payload"], {}),
                "status": r["status"], "attempts": r["attempts"],
                "max_attempts": r["max_attempts"], "lease_until": _s(r["lease_until"]),
                "deadline_at": _s(r["deadline_at"]),
                "result": _loads(r["result"], None), "error": r["error"] or None,
                "priority": r["priority"], "queued_at": _s(r["queued_at"]),
                "updated_at": _s(r["updated_at"]), "source": r["source"],
                "device_id": r["device_id"] or None, "worker_id": r["worker_id"] or None,
                "progress": self.progress.get(r["id"])}

    def submit_job(self, kind, payload, priority=0, source="", max_attempts=3,
                   deadline_at=None, status="queued"):
        payload = payload if isinstance(payload, dict) else {}
        return self.q.submit(kind, json.dumps(payload), int(priority), source or "",
                             int(max_attempts or 3), _ms(deadline_at),
                             str(payload.get("device_id") or ""),
                             str(payload.get("model_id") or payload.get("model") or ""),
                             _ms(self.clock()), status)

    def get_job(self, job_id):
        r = self.q.get(job_id)
        return None if r is None else self._job(r)

    def _online(self) -> list[str]:
        with self._lock:
            return [d for d, v in self.devices.items() if v.get("status") == "online"]

    def claim_job(self, worker_id, kinds, lease_s, worker_device="", device_max_concurrency=1,
                  check_online=True):
        limits = {}
        with self._lock:
            # GPU engine devices admit as many jobs as their batching capacity
            for dev, d in self.devices.items():
                cap = (d.get("tags") or {}).get("capacity")
                if cap:
                    limits[dev] = int(cap)
            for dev, lim in self.device_limits.items():
                if lim.get("max_concurrency"):
                    limits[dev] = int(lim["max_concurrency"])
        r = self.q.claim(worker_id, list(kinds or []), worker_device or "",
                         self._online() if check_online else [], bool(check_online),
                         int(device_max_concurrency or 0), limits, int(lease_s * 1000),
                         _ms(self.clock()))
        if r is None:
            return None
        j = self._job(r)
        j["attempt_id"] = r["attempt_id"]
        return j

    def heartbeat(self, job_id, worker_id, extend_s, token="", progress=None):
        """Extend the lease; a ``progress`` dict (tokens generated so far, ...)
        from the lease owner is kept with the job and wakes job streams."""
        ok = self.q.heartbeat(job_id, worker_id, token or "", int(extend_s * 1000),
                              _ms(self.clock()))
        if ok and isinstance(progress, dict):
            with self._lock:
                self.progress[job_id] = progress
            self.q.notify_change()
        return ok

    def complete_job(self, job_id, worker_id, result, metrics, token=""):
        ok = self.q.complete(job_id, worker_id, token or "", json.dumps(result or {}),
                             json.dumps(metrics or {}), _ms(self.clock()))
        if ok:
            with self._lock:
                self.progress.pop(job_id, None)
        return ok

    def fail_job(self, job_id, worker_id, error, metrics, token=""):
        st = self.q.fail(job_id, worker_id, token or "", error or "", json.dumps(metrics or {}),
                         _ms(self.clock()))
        if st:
            with self._lock:
                self.progress.pop(job_id, None)
        return st or None

    def release_device_leases(self, device_id):
        return self.q.release_device(device_id, _ms(self.clock()))

    def expire_deadlines(self):
        return self.q.expire_deadlines(_ms(self.clock()))

    def sweep_exhausted(self):
        return 0      # the native queue retires attempt-capped rows inside claim()

    def purge_jobs(self, older_than_s):
        return self.q.purge_finished(_ms(self.clock() - older_than_s))

    def job_counts(self):
        return dict(self.q.counts())

    def running_jobs(self, limit=10):
        return [self._job(r) for r in self.q.list("running", limit)]

    def list_jobs(self, status="", limit=50):
        return [self._job(r) for r in self.q.list(status, limit)]

    def stuck_jobs(self):
        return self.q.stuck(_ms(self.clock()))

    def failed_jobs_since(self, since, min_attempts):
        out = []
        for r in self.q.list("error", 500):
            if r["updated_at"] >= _ms(since) and r["attempts"] >= min_attempts:
                out.append(self._job(r))
        return out

    def job_attempts(self, job_id):
        return [{"id": a["id"], "job_id": a["job_id"], "worker_id": a["worker_id"],
                 "status": a["status"], "error": a["error"] or None,
                 "metrics": _loads(a["metrics"], {}), "started_at": _s(a["started_at"]),
                 "finished_at": _s(a["finished_at"])} for a in self.q.attempts(job_id)]

    def active_jobs_on(self, device_id):
        return self.q.active_on(device_id or "")

    def job_version(self):
        return self.q.version

    def wait_job_change(self, since, timeout_s):
        return self.q.wait_change(int(since), int(timeout_s * 1000))

    # -------------------------------------------------------------- devices --
    def upsert_device(self, device_id, name="", platform="", arch="", host="", tags=None,
                      status="online", merge_tags=False):
        t = self.clock()
        with self._lock:
            d = self.devices.get(device_id)
            if d is None:
                d = {"id": device_id, "created_at": t, "tags": {}}
                self.devices[device_id] = d
            d.update(name=name or d.get("name", ""), platform=platform or d.get("platform", ""),
                     arch=arch or d.get("arch", ""), host=host or d.get("host", ""),
                     status=status, updated_at=t)
            if status == "online":
                d["last_seen"] = t
            if tags is not None:
                d["tags"] = {**d.get("tags", {}), **tags} if merge_tags else dict(tags)

    def get_device(self, device_id):
        with self._lock:
            d = self.devices.get(device_id)
            return None if d is None else json.loads(json.dumps(d))

    def list_devices(self):
        with self._lock:
            return [json.loads(json.dumps(d)) for d in sorted(self.devices.values(),
                                                              key=lambda x: x["id"])]

    def set_device_status(self, device_id, status, tags=None):
        with self._lock:
            d = self.devices.get(device_id)
            if d is None:
                return False
            d["status"] = status
            d["updated_at"] = self.clock()
            if status == "online":
                d["last_seen"] = d["updated_at"]
            if tags:
                d["tags"] = {**d.get("tags", {}), **tags}
            return True

    def delete_devices(self, prefix):
        with self._lock:
            ids = [k for k in self.devices if k.startswith(prefix)]
            for k in ids:
                del self.devices[k]
                for key in [key for key in self.device_models if key[0] == k]:
                    del self.device_models[key]
            return len(ids)

    def insert_device_metrics(self, device_id, metrics):
        with self._lock:
            self.device_metrics.append({"device_id": device_id, "ts": self.clock(),
                                        "notes": metrics})
            del self.device_metrics[:-1000]

    # --------------------------------------------------------------- models --
    _MODEL_FIELDS = ("provider", "family", "kind", "params_b", "context_k", "size_gb", "quant",
                     "status", "tier", "thinking", "meta")

    def upsert_model(self, model_id, **fields):
        with self._lock:
            m = self.models.setdefault(model_id, {"id": model_id, "provider": "local",
                                                  "kind": "chat", "status": "active"})
            for k, v in fields.items():
                if k in self._MODEL_FIELDS and v is not None:
                    m[k] = v
            m["updated_at"] = self.clock()

    def get_model(self, model_id):
        with self._lock:
            m = self.models.get(model_id)
            return None if m is None else dict(m)

    def list_models(self, provider=None):
        with self._lock:
            return [dict(m) for m in self.models.values()
                    if provider is None or m.get("provider") == provider]

    def set_pricing(self, model_id, price_in_1m, price_out_1m):
        with self._lock:
            self.pricing[model_id] = (float(price_in_1m or 0), float(price_out_1m or 0))

    def get_pricing(self, model_id):
        with self._lock:
            return self.pricing.get(model_id)

    def upsert_device_model(self, device_id, model_id, available=True, max_context_k=None,
                            meta=None):
        with self._lock:
            self.device_models[(device_id, model_id)] = {
                "device_id": device_id, "model_id": model_id, "available": bool(available),
                "max_context_k": max_context_k, "meta": meta or {}, "updated_at": self.clock()}

    def list_device_models(self, device_id=None, available_only=False):
        with self._lock:
            return [dict(v) for (d, _), v in self.device_models.items()
                    if (device_id is None or d == device_id)
                    and (not available_only or v["available"])]

    def mark_absent_models(self, device_id, present):
        keep = set(present)
        n = 0
        with self._lock:
            for (d, m), v in self.device_models.items():
                if d == device_id and m not in keep and v["available"]:
                    v["available"] = False
                    n += 1
        return n

    # ------------------------------------------------ benchmarks / limits ----
    def insert_benchmark(self, device_id, model_id, task_type, tokens_in, tokens_out,
                         latency_ms, tps, meta=None, ok=True):
        with self._lock:
            self.benchmarks.append({
                "id": str(uuid.uuid4()), "device_id": device_id, "model_id": model_id,
                "task_type": task_type, "tokens_in": int(tokens_in or 0),
                "tokens_out": int(tokens_out or 0), "latency_ms": int(latency_ms or 0),
                "tps": float(tps or 0), "meta": meta or {}, "ok": bool(ok),
                "created_at": self.clock()})
            del self.benchmarks[:-5000]

    def list_benchmarks(self, limit=20):
        with self._lock:
            return [dict(b) for b in reversed(self.benchmarks[-limit:])]

    def latest_benchmark(self, model_id, task_type, device_id=None):
        with self._lock:
            for b in reversed(self.benchmarks):
                if b["model_id"] == model_id and b["task_type"] == task_type and \
                        (device_id is None or b["device_id"] == device_id):
                    return dict(b)
        return None

    def upsert_device_limits(self, device_id, spec):
        with self._lock:
            self.device_limits[device_id] = {**dict(spec), "device_id": device_id,
                                             "updated_at": self.clock()}

    def get_device_limits(self, device_id):
        with self._lock:
            v = self.device_limits.get(device_id)
            return None if v is None else dict(v)

    # ---------------------------------------------------------------- costs --
    def calculate_job_cost(self, model_id, tokens_in, tokens_out):
        """calculate_job_cost() plpgsql (02_v2_improvements.sql:55-79)."""
        p = self.get_pricing(model_id)
        if p is None:
            return 0.0
        return (tokens_in * p[0] + tokens_out * p[1]) / 1_000_000.0

    def insert_cost(self, job_id, model_id, provider, tokens_in, tokens_out, cost_usd):
        with self._lock:
            self.costs.append({"id": str(uuid.uuid4()), "job_id": job_id, "model_id": model_id,
                               "provider": provider, "tokens_in": int(tokens_in),
                               "tokens_out": int(tokens_out), "cost_usd": float(cost_usd),
                               "created_at": self.clock()})

    def cost_summary(self, since):
        by: dict[str, dict] = {}
        total, jobs = 0.0, 0
        with self._lock:
            for c in self.costs:
                if c["created_at"] < since:
                    continue
                p = by.setdefault(c["provider"], {"provider": c["provider"], "cost_usd": 0.0,
                                                  "jobs": 0, "tokens_in": 0, "tokens_out": 0})
                p["cost_usd"] += c["cost_usd"]
                p["jobs"] += 1
                p["tokens_in"] += c["tokens_in"]
                p["tokens_out"] += c["tokens_out"]
                total += c["cost_usd"]
                jobs += 1
        return {"total_cost": total, "total_jobs": jobs,
                "by_provider": sorted(by.values(), key=lambda x: -x["cost_usd"])}

    def cost_top_models(self, since, limit=10):
        agg: dict[str, dict] = {}
        with self._lock:
            for c in self.costs:
                if c["created_at"] < since:
                    continue
                a = agg.setdefault(c["model_id"], {"model": c["model_id"], "cost_usd": 0.0,
                                                   "requests": 0})
                a["cost_usd"] += c["cost_usd"]
                a["requests"] += 1
        return sorted(agg.values(), key=lambda x: -x["cost_usd"])[:limit]

    # --------------------------------------------------- rankings / stats ----
    def upsert_model_ranking(self, model_id, **fields):
        with self._lock:
            r = self.rankings.setdefault(model_id, {"model_id": model_id})
            r.update({k: v for k, v in fields.items() if v is not None})
            r["updated_at"] = self.clock()

    def list_model_rankings(self):
        with self._lock:
            return [dict(r) for r in self.rankings.values()]

    def _stat(self, model_id):
        # column names of model_stats (db/migrations/05_chat_rankings.sql)
        return self.stats.setdefault(model_id, {
            "model_id": model_id, "total_requests": 0, "total_tokens_in": 0,
            "total_tokens_out": 0, "total_cost_usd": 0.0, "avg_duration_ms": 0.0,
            "error_count": 0, "feedback_positive": 0, "feedback_negative": 0,
            "last_used_at": None})

    def update_model_stats(self, model_id, tokens_in, tokens_out, latency_ms, cost, ok):
        """Running-average upsert (handlers.go:3147-3171)."""
        with self._lock:
            s = self._stat(model_id)
            n = s["total_requests"]
            s["avg_duration_ms"] = (s["avg_duration_ms"] * n + latency_ms) / (n + 1)
            s["total_requests"] = n + 1
            if not ok:
                s["error_count"] += 1
            s["total_tokens_in"] += int(tokens_in)
            s["total_tokens_out"] += int(tokens_out)
            s["total_cost_usd"] += float(cost)
            s["last_used_at"] = self.clock()

    def feedback(self, model_id, good):
        with self._lock:
            s = self._stat(model_id)
            s["feedback_positive" if good else "feedback_negative"] += 1
            return True

    def model_stats(self):
        with self._lock:
            out = []
            for s in self.stats.values():
                d = dict(s)
                n = d["total_requests"]
                # generated columns of model_stats
                d["success_rate"] = round((n - d["error_count"]) * 100.0 / n, 2) if n else 0.0
                d["avg_cost_per_request"] = (d["total_cost_usd"] / n) if n else 0.0
                out.append(d)
            return out

    def device_stats_7d(self, device_id):
        """v_device_stats (04_smart_routing.sql:71-94) from job attempts, counted
        in the native queue (the dashboard asks per device on every poll)."""
        s = self.q.device_stats(device_id, _ms(self.clock() - 7 * 86400))
        total, done = s["total"], s["done"]
        return {"total_jobs_7d": total, "done_jobs_7d": done,
                "success_rate": (done / total) if total else 0.0,
                "avg_latency_ms": int(s["ms_sum"] / s["ms_n"]) if s["ms_n"] else 0}

    def kind_counts(self, prefix):
        """{status: jobs} of the jobs whose kind starts with ``prefix``."""
        return dict(self.q.kind_counts(prefix))
