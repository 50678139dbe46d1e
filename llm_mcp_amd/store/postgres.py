"""PostgreSQL store: the reference's durable control-plane state
(db/init/01_core.sql + db/migrations/02..05) behind the ``Store`` interface,
over the in-tree wire-protocol client (store/pgwire.py).

* ``migrate()`` applies store/schema.sql idempotently at startup (the
  reference required migrations 02-05 to be applied by hand).
* ``claim_job`` is the reference's lease claim (handlers.go:173-293): one
  transaction, ``running_per_device`` CTE counting *live* leases,
  ``FOR UPDATE SKIP LOCKED LIMIT 1``, attempts+1, lease, ``job_attempts``
  row -- plus the fixes of the native queue: expired leases are reclaimable,
  deadlines/attempt caps are enforced, a lease token guards heartbeat /
  complete / fail, and the gRPC path gets the same concurrency check.
* job status changes NOTIFY ``job_update`` (trigger); ``wait_job_change``
  LISTENs on a dedicated connection (the SSE stream's wake-up,
  handlers.go:514-545).

Semantics are kept identical to MemoryStore (store/memory.py); all
timestamps crossing the interface are epoch seconds.
"""
from __future__ import annotations

import json
import os
import threading
import time

from .pgwire import Connection, Pool

_SCHEMA = os.path.join(os.path.dirname(__file__), "schema.sql")

_JOB_COLS = ("id::text AS id, kind, payload, status, attempts, max_attempts, lease_until, "
             "deadline_at, result, error, priority, queued_at, updated_at, source, device_id, "
             "worker_id, progress")


def _job(r: dict | None) -> dict | None:
    if r is None:
        return None
    d = dict(r)
    d["payload"] = d.get("payload") or {}
    d["source"] = d.get("source") or ""
    d["error"] = d.get("error") or None
    return d


class PostgresStore:
    backend = "postgres"

    def __init__(self, dsn: str, pool_size: int = 8, migrate: bool = True):
        self.dsn = dsn
        self.pool = Pool(dsn, pool_size)
        if migrate:
            self.migrate()
        self._version = 0
        self._cv = threading.Condition()
        self._listener_stop = threading.Event()
        self._listener = threading.Thread(target=self._listen, daemon=True, name="pg-listen")
        self._listener.start()

    # ------------------------------------------------------------ plumbing --
    def migrate(self) -> None:
        with open(_SCHEMA) as f:
            script = f.read()
        with self.pool.conn() as c:
            c.simple("SELECT pg_advisory_lock(727001)")   # one migrator at a time
            try:
                c.simple(script)
            finally:
                c.simple("SELECT pg_advisory_unlock(727001)")

    def _q(self, sql: str, *params) -> list[dict]:
        with self.pool.conn() as c:
            return c.query(sql, *params)

    def _one(self, sql: str, *params) -> dict | None:
        r = self._q(sql, *params)
        return r[0] if r else None

    def _n(self, sql: str, *params) -> int:
        with self.pool.conn() as c:
            return c.rowcount(sql, *params)

    def _listen(self):
        while not self._listener_stop.is_set():
            try:
                c = Connection(self.dsn)
                c.listen("job_update")
                while not self._listener_stop.is_set():
                    if c.wait_notify(1.0):
                        self._bump()
            except Exception:
                time.sleep(1.0)   # reconnect; pollers fall back to their timeout
                self._bump()

    def _bump(self):
        with self._cv:
            self._version += 1
            self._cv.notify_all()

    def close(self):
        self._listener_stop.set()
        self.pool.close()

    def ping(self) -> bool:
        try:
            return self._one("SELECT 1 AS ok")["ok"] == 1
        except Exception:
            return False

    # ---------------------------------------------------------------- jobs --
    def submit_job(self, kind, payload, priority=0, source="", max_attempts=3,
                   deadline_at=None, status="queued"):
        payload = payload if isinstance(payload, dict) else {}
        r = self._one(
            "INSERT INTO jobs (kind, payload, priority, source, max_attempts, deadline_at, "
            "status, device_id) VALUES ($1, $2::jsonb, $3, $4, $5, to_timestamp($6), $7, "
            "NULLIF($8, '')) RETURNING id::text AS id",
            kind, payload, int(priority), source or "", int(max_attempts or 3), deadline_at,
            status, str(payload.get("device_id") or ""))
        return r["id"]

    def get_job(self, job_id):
        try:
            return _job(self._one(f"SELECT {_JOB_COLS} FROM jobs WHERE id = $1::uuid", job_id))
        except Exception:
            return None

    def _limits(self, c) -> dict[str, int]:
        lim = {}
        for r in c.query("SELECT id, (tags->>'capacity')::int AS cap FROM devices "
                         "WHERE tags ? 'capacity'"):
            if r["cap"]:
                lim[r["id"]] = r["cap"]
        for r in c.query("SELECT device_id, max_concurrency FROM device_limits "
                         "WHERE max_concurrency IS NOT NULL AND max_concurrency > 0"):
            lim[r["device_id"]] = r["max_concurrency"]
        return lim

    def claim_job(self, worker_id, kinds, lease_s, worker_device="", device_max_concurrency=1,
                  check_online=True):
        PIN = "NULLIF(j.payload->>'device_id', '')"   # noqa: N806 (SQL fragment)
        # The claim transaction locks exactly one row, by SKIP LOCKED: expired
        # deadlines and attempt-capped rows are filtered out here and retired
        # by the maintenance sweep (expire_deadlines / sweep_exhausted, also
        # SKIP LOCKED), so concurrent claimers never queue on each other.
        with self.pool.conn() as c, c.transaction():
            limits = self._limits(c)
            r = c.one(
                f"""
                WITH running_per_device AS (
                  SELECT device_id, COUNT(*) AS n FROM jobs
                  WHERE status = 'running' AND lease_until >= now() AND device_id IS NOT NULL
                  GROUP BY device_id
                ), cand AS (
                  -- only the submitter's pin (payload device_id) restricts
                  -- placement; jobs.device_id is where the job last ran, so a
                  -- requeued / lease-lapsed job may move to any device
                  SELECT j.id, COALESCE({PIN}, NULLIF($3, '')) AS place
                  FROM jobs j
                  LEFT JOIN running_per_device r
                         ON r.device_id = COALESCE({PIN}, NULLIF($3, ''))
                  LEFT JOIN devices d ON d.id = {PIN}
                  WHERE (j.status = 'queued' OR (j.status = 'running' AND j.lease_until < now()))
                    AND j.attempts < j.max_attempts
                    AND (j.deadline_at IS NULL OR j.deadline_at >= now())
                    AND (cardinality($2::text[]) = 0 OR j.kind = ANY($2::text[]))
                    AND ({PIN} IS NULL OR $3 = '' OR {PIN} = $3)
                    AND (NOT $5 OR {PIN} IS NULL OR d.status = 'online')
                    AND (COALESCE({PIN}, NULLIF($3, '')) IS NULL
                         OR COALESCE(($6::jsonb ->> COALESCE({PIN}, $3))::int, $4) <= 0
                         OR COALESCE(r.n, 0) <
                            COALESCE(($6::jsonb ->> COALESCE({PIN}, $3))::int, $4))
                  ORDER BY j.priority DESC, j.queued_at ASC
                  FOR UPDATE OF j SKIP LOCKED
                  LIMIT 1
                ), closed AS (
                  UPDATE job_attempts a SET status = 'lease_expired', finished_at = now()
                  FROM jobs j, cand WHERE j.id = cand.id AND a.id = j.lease_token
                    AND a.status = 'running'
                )
                UPDATE jobs SET status = 'running', attempts = jobs.attempts + 1,
                       lease_until = now() + make_interval(secs => $7),
                       worker_id = $1, device_id = cand.place,
                       lease_token = gen_random_uuid(), updated_at = now()
                FROM cand WHERE jobs.id = cand.id
                RETURNING {", ".join("jobs." + x.strip() for x in _JOB_COLS.split(", "))},
                          jobs.lease_token::text AS attempt_id
                """,
                worker_id, list(kinds or []), worker_device or "",
                int(device_max_concurrency or 0), bool(check_online), limits, float(lease_s))
            if r is None:
                return None
            c.query("INSERT INTO job_attempts (id, job_id, worker_id, status) "
                    "VALUES ($1::uuid, $2::uuid, $3, 'running')",
                    r["attempt_id"], r["id"], worker_id)
        return _job(r)

    _OWNS = ("status = 'running' AND (($3 <> '' AND lease_token::text = $3) OR "
             "($3 = '' AND worker_id = $2))")

    def heartbeat(self, job_id, worker_id, extend_s, token="", progress=None):
        # a progress change NOTIFYs job_update (trigger), waking job streams
        return self._n(
            f"UPDATE jobs SET lease_until = now() + make_interval(secs => $4), "
            f"progress = COALESCE($5::jsonb, progress), "
            f"updated_at = now() WHERE id = $1::uuid AND {self._OWNS}",
            job_id, worker_id, token or "", float(extend_s),
            progress if isinstance(progress, dict) else None) == 1

    def complete_job(self, job_id, worker_id, result, metrics, token=""):
        with self.pool.conn() as c, c.transaction():
            r = c.one(f"UPDATE jobs SET status = 'done', result = $4::jsonb, lease_until = NULL, "
                      f"updated_at = now() WHERE id = $1::uuid AND {self._OWNS} "
                      f"RETURNING lease_token::text AS tok", job_id, worker_id, token or "",
                      result or {})
            if r is None:
                return False
            c.query("UPDATE job_attempts SET status = 'done', finished_at = now(), "
                    "metrics = $2::jsonb WHERE id = $1::uuid", r["tok"], metrics or {})
        return True

    def fail_job(self, job_id, worker_id, error, metrics, token=""):
        with self.pool.conn() as c, c.transaction():
            tok = c.one(f"SELECT lease_token::text AS tok FROM jobs WHERE id = $1::uuid "
                        f"AND {self._OWNS} FOR UPDATE", job_id, worker_id, token or "")
            if tok is None:
                return None
            # a requeued job drops its placement (back to the submitter's pin)
            r = c.one("UPDATE jobs SET error = $2, lease_until = NULL, lease_token = NULL, "
                      "updated_at = now(), status = CASE WHEN attempts < max_attempts "
                      "THEN 'queued' ELSE 'error' END, device_id = CASE WHEN attempts < "
                      "max_attempts THEN NULLIF(payload->>'device_id', '') ELSE device_id END "
                      "WHERE id = $1::uuid "
                      "RETURNING status, $3::text AS tok", job_id, error or "", tok["tok"])
            if r is None:
                return None
            c.query("UPDATE job_attempts SET status = 'error', error = $2, finished_at = now(), "
                    "metrics = $3::jsonb WHERE id = $1::uuid", r["tok"], error or "",
                    metrics or {})
        return r["status"]

    def release_device_leases(self, device_id):
        return self._n("UPDATE jobs SET lease_until = to_timestamp(0), updated_at = now() "
                       "WHERE status = 'running' AND device_id = $1", device_id)

    def expire_deadlines(self):
        """Retire jobs past deadline_at (queued, or running with a lapsed
        lease: a live lease finishes its attempt).  Rows another transaction
        holds (a claim in progress) are skipped, not waited for."""
        return self._n("UPDATE jobs SET status = 'error', error = 'deadline_exceeded', "
                       "lease_until = NULL, lease_token = NULL, updated_at = now() "
                       "WHERE id IN (SELECT id FROM jobs WHERE status IN ('queued', 'running') "
                       "AND deadline_at IS NOT NULL AND deadline_at < now() "
                       "AND (status = 'queued' OR lease_until < now()) "
                       "FOR UPDATE SKIP LOCKED)")

    def sweep_exhausted(self):
        """Queued (or lease-lapsed) rows whose attempts reached max_attempts ->
        error 'attempts_exhausted' (they can never be claimed again)."""
        return self._n("UPDATE jobs SET status = 'error', error = 'attempts_exhausted', "
                       "lease_until = NULL, lease_token = NULL, updated_at = now() "
                       "WHERE id IN (SELECT id FROM jobs WHERE attempts >= max_attempts "
                       "AND (status = 'queued' OR (status = 'running' AND lease_until < now())) "
                       "FOR UPDATE SKIP LOCKED)")

    def purge_jobs(self, older_than_s):
        return self._n("DELETE FROM jobs WHERE status IN ('done', 'error') "
                       "AND updated_at < now() - make_interval(secs => $1)", float(older_than_s))

    def job_counts(self):
        out = {"queued": 0, "running": 0, "done": 0, "error": 0}
        for r in self._q("SELECT status, COUNT(*)::int AS n FROM jobs GROUP BY status"):
            out[r["status"]] = r["n"]
        return out

    def kind_counts(self, prefix):
        """{status: jobs} of the jobs whose kind starts with ``prefix``."""
        return {r["status"]: r["n"] for r in self._q(
            "SELECT status, COUNT(*)::int AS n FROM jobs WHERE starts_with(kind, $1) "
            "GROUP BY status", prefix)}

    def running_jobs(self, limit=10):
        return self.list_jobs("running", limit)

    def list_jobs(self, status="", limit=50):
        lim = int(limit) if limit else 1_000_000
        return [_job(r) for r in self._q(
            f"SELECT {_JOB_COLS} FROM jobs WHERE ($1 = '' OR status = $1) "
            f"ORDER BY updated_at DESC LIMIT $2", status or "", lim)]

    def stuck_jobs(self):
        return self._one("SELECT COUNT(*)::int AS n FROM jobs WHERE status = 'running' "
                         "AND lease_until < now()")["n"]

    def failed_jobs_since(self, since, min_attempts):
        return [_job(r) for r in self._q(
            f"SELECT {_JOB_COLS} FROM jobs WHERE status = 'error' AND updated_at >= "
            f"to_timestamp($1) AND attempts >= $2 ORDER BY updated_at DESC LIMIT 500",
            float(since), int(min_attempts))]

    def job_attempts(self, job_id):
        return [{**r, "error": r["error"] or None, "metrics": r["metrics"] or {}}
                for r in self._q("SELECT id::text AS id, job_id::text AS job_id, worker_id, "
                                 "status, error, metrics, started_at, finished_at "
                                 "FROM job_attempts WHERE job_id = $1::uuid ORDER BY started_at",
                                 job_id)]

    def active_jobs_on(self, device_id):
        return self._one("SELECT COUNT(*)::int AS n FROM jobs WHERE device_id = $1 "
                         "AND status IN ('queued', 'running')", device_id)["n"]

    def job_version(self):
        return self._version

    def wait_job_change(self, since, timeout_s):
        deadline = time.monotonic() + timeout_s
        with self._cv:
            while self._version <= since:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                self._cv.wait(left)
            return self._version

    # -------------------------------------------------------------- devices --
    def upsert_device(self, device_id, name="", platform="", arch="", host="", tags=None,
                      status="online", merge_tags=False):
        self._q(
            "INSERT INTO devices (id, name, platform, arch, host, tags, status, last_seen) "
            "VALUES ($1, $2, $3, $4, $5, COALESCE($6::jsonb, '{}'), $7, "
            "CASE WHEN $7 = 'online' THEN now() END) "
            "ON CONFLICT (id) DO UPDATE SET "
            "name = COALESCE(NULLIF(EXCLUDED.name, ''), devices.name), "
            "platform = COALESCE(NULLIF(EXCLUDED.platform, ''), devices.platform), "
            "arch = COALESCE(NULLIF(EXCLUDED.arch, ''), devices.arch), "
            "host = COALESCE(NULLIF(EXCLUDED.host, ''), devices.host), "
            "tags = CASE WHEN $6::jsonb IS NULL THEN devices.tags "
            "            WHEN $8 THEN devices.tags || $6::jsonb ELSE $6::jsonb END, "
            "status = EXCLUDED.status, updated_at = now(), "
            "last_seen = CASE WHEN EXCLUDED.status = 'online' THEN now() "
            "                 ELSE devices.last_seen END",
            device_id, name or "", platform or "", arch or "", host or "", tags, status,
            bool(merge_tags))

    _DEV = ("id, name, platform, arch, host, tags, status, last_seen, created_at, updated_at")

    def get_device(self, device_id):
        return self._one(f"SELECT {self._DEV} FROM devices WHERE id = $1", device_id)

    def list_devices(self):
        return self._q(f"SELECT {self._DEV} FROM devices ORDER BY id")

    def set_device_status(self, device_id, status, tags=None):
        return self._n("UPDATE devices SET status = $2, updated_at = now(), "
                       "last_seen = CASE WHEN $2 = 'online' THEN now() ELSE last_seen END, "
                       "tags = CASE WHEN $3::jsonb IS NULL THEN tags ELSE tags || $3::jsonb END "
                       "WHERE id = $1", device_id, status, tags or None) == 1

    def delete_devices(self, prefix):
        return self._n("DELETE FROM devices WHERE starts_with(id, $1)", prefix)

    def insert_device_metrics(self, device_id, metrics):
        m = metrics or {}
        self._q("INSERT INTO device_metrics (device_id, cpu_pct, mem_used_mb, mem_total_mb, "
                "gpu_name, vram_used_mb, vram_total_mb, tps, latency_ms, notes) "
                "SELECT $1, $2, $3, $4, $5, $6, $7, $8, $9, $10::jsonb "
                "WHERE EXISTS (SELECT 1 FROM devices WHERE id = $1)",
                device_id, m.get("cpu_pct"), m.get("mem_used_mb"), m.get("mem_total_mb"),
                m.get("gpu_name"), m.get("vram_used_mb"), m.get("vram_total_mb"), m.get("tps"),
                m.get("latency_ms"), m)

    # --------------------------------------------------------------- models --
    _MODEL_FIELDS = ("provider", "family", "kind", "params_b", "context_k", "size_gb", "quant",
                     "status", "tier", "thinking", "meta")

    def upsert_model(self, model_id, **fields):
        f = {k: v for k, v in fields.items() if k in self._MODEL_FIELDS and v is not None}
        cols = ["id"] + list(f)
        vals = [model_id] + [f[k] for k in f]
        ph = ", ".join(f"${i + 1}" + ("::jsonb" if c == "meta" else "")
                       for i, c in enumerate(cols))
        upd = ", ".join(f"{c} = EXCLUDED.{c}" for c in f)
        self._q(f"INSERT INTO models ({', '.join(cols)}) VALUES ({ph}) ON CONFLICT (id) DO "
                + (f"UPDATE SET {upd}, updated_at = now()" if upd else
                   "UPDATE SET updated_at = now()"), *vals)

    _MODEL = ("id, provider, family, kind, params_b, context_k, size_gb, quant, status, tier, "
              "thinking, meta, updated_at")

    def get_model(self, model_id):
        return self._one(f"SELECT {self._MODEL} FROM models WHERE id = $1", model_id)

    def list_models(self, provider=None):
        return self._q(f"SELECT {self._MODEL} FROM models WHERE ($1::text IS NULL OR "
                       f"provider = $1) ORDER BY id", provider)

    def set_pricing(self, model_id, price_in_1m, price_out_1m):
        self._q("INSERT INTO model_pricing (model_id, price_in_1m, price_out_1m) "
                "VALUES ($1, $2, $3) ON CONFLICT (model_id) DO UPDATE SET "
                "price_in_1m = EXCLUDED.price_in_1m, price_out_1m = EXCLUDED.price_out_1m, "
                "updated_at = now()", model_id, float(price_in_1m or 0), float(price_out_1m or 0))

    def get_pricing(self, model_id):
        r = self._one("SELECT price_in_1m, price_out_1m FROM model_pricing WHERE model_id = $1",
                      model_id)
        return None if r is None else (r["price_in_1m"] or 0.0, r["price_out_1m"] or 0.0)

    def upsert_device_model(self, device_id, model_id, available=True, max_context_k=None,
                            meta=None):
        self._q("INSERT INTO device_models (device_id, model_id, available, max_context_k, meta) "
                "VALUES ($1, $2, $3, $4, $5::jsonb) ON CONFLICT (device_id, model_id) DO UPDATE "
                "SET available = EXCLUDED.available, max_context_k = EXCLUDED.max_context_k, "
                "meta = EXCLUDED.meta, updated_at = now()",
                device_id, model_id, bool(available), max_context_k, meta or {})

    def list_device_models(self, device_id=None, available_only=False):
        rows = self._q("SELECT device_id, model_id, available, max_context_k, meta, updated_at "
                       "FROM device_models WHERE ($1::text IS NULL OR device_id = $1) "
                       "AND (NOT $2 OR available)", device_id, bool(available_only))
        for r in rows:
            r["meta"] = r["meta"] or {}
        return rows

    def mark_absent_models(self, device_id, present):
        return self._n("UPDATE device_models SET available = FALSE, updated_at = now() "
                       "WHERE device_id = $1 AND available AND NOT (model_id = ANY($2::text[]))",
                       device_id, list(present))

    # ------------------------------------------------ benchmarks / limits ----
    def insert_benchmark(self, device_id, model_id, task_type, tokens_in, tokens_out,
                         latency_ms, tps, meta=None, ok=True):
        self._q("INSERT INTO benchmarks (device_id, model_id, task_type, tokens_in, tokens_out, "
                "latency_ms, tps, meta, ok) VALUES ($1, $2, $3, $4, $5, $6, $7, $8::jsonb, $9)",
                device_id, model_id, task_type, int(tokens_in or 0), int(tokens_out or 0),
                int(latency_ms or 0), float(tps or 0), meta or {}, bool(ok))

    _BENCH = ("id::text AS id, device_id, model_id, task_type, tokens_in, tokens_out, "
              "latency_ms, tps, meta, ok, created_at")

    def list_benchmarks(self, limit=20):
        return self._q(f"SELECT {self._BENCH} FROM benchmarks ORDER BY created_at DESC "
                       f"LIMIT $1", int(limit))

    def latest_benchmark(self, model_id, task_type, device_id=None):
        return self._one(f"SELECT {self._BENCH} FROM benchmarks WHERE model_id = $1 AND "
                         f"task_type = $2 AND ($3::text IS NULL OR device_id = $3) "
                         f"ORDER BY created_at DESC LIMIT 1", model_id, task_type, device_id)

    def upsert_device_limits(self, device_id, spec):
        s = dict(spec or {})
        self._q("INSERT INTO device_limits (device_id, ram_gb, vram_gb, max_params_b, "
                "max_size_gb, max_context_k, allow_models, deny_models, max_concurrency, spec) "
                "VALUES ($1, $2, $3, $4, $5, $6, $7::jsonb, $8::jsonb, $9, $10::jsonb) "
                "ON CONFLICT (device_id) DO UPDATE SET ram_gb = EXCLUDED.ram_gb, "
                "vram_gb = EXCLUDED.vram_gb, max_params_b = EXCLUDED.max_params_b, "
                "max_size_gb = EXCLUDED.max_size_gb, max_context_k = EXCLUDED.max_context_k, "
                "allow_models = EXCLUDED.allow_models, deny_models = EXCLUDED.deny_models, "
                "max_concurrency = EXCLUDED.max_concurrency, spec = EXCLUDED.spec, "
                "updated_at = now()",
                device_id, s.get("ram_gb"), s.get("vram_gb"), s.get("max_params_b"),
                s.get("max_size_gb"), s.get("max_context_k"),
                json.dumps(s.get("allow_models")) if s.get("allow_models") is not None else None,
                json.dumps(s.get("deny_models")) if s.get("deny_models") is not None else None,
                s.get("max_concurrency"), s)

    def get_device_limits(self, device_id):
        r = self._one("SELECT spec, updated_at FROM device_limits WHERE device_id = $1",
                      device_id)
        if r is None:
            return None
        return {**(r["spec"] or {}), "device_id": device_id, "updated_at": r["updated_at"]}

    # ---------------------------------------------------------------- costs --
    def calculate_job_cost(self, model_id, tokens_in, tokens_out):
        return float(self._one("SELECT calculate_job_cost($1, $2, $3) AS c", model_id,
                               int(tokens_in), int(tokens_out))["c"] or 0.0)

    def insert_cost(self, job_id, model_id, provider, tokens_in, tokens_out, cost_usd):
        self._q("INSERT INTO llm_costs (job_id, model_id, provider, tokens_in, tokens_out, "
                "cost_usd) VALUES ($1::uuid, $2, $3, $4, $5, $6)", job_id, model_id, provider,
                int(tokens_in), int(tokens_out), float(cost_usd))

    def cost_summary(self, since):
        rows = self._q("SELECT provider, SUM(cost_usd)::float8 AS cost_usd, COUNT(*)::int AS jobs, "
                       "SUM(tokens_in)::int AS tokens_in, SUM(tokens_out)::int AS tokens_out "
                       "FROM llm_costs WHERE created_at >= to_timestamp($1) GROUP BY provider "
                       "ORDER BY 2 DESC", float(since))
        return {"total_cost": sum(r["cost_usd"] for r in rows),
                "total_jobs": sum(r["jobs"] for r in rows), "by_provider": rows}

    def cost_top_models(self, since, limit=10):
        return self._q("SELECT model_id AS model, SUM(cost_usd)::float8 AS cost_usd, "
                       "COUNT(*)::int AS requests FROM llm_costs WHERE created_at >= "
                       "to_timestamp($1) GROUP BY model_id ORDER BY 2 DESC LIMIT $2",
                       float(since), int(limit))

    # --------------------------------------------------- rankings / stats ----
    _RANK_FIELDS = ("provider", "display_name", "category_scores", "context_k", "price_in_1m",
                    "price_out_1m", "modalities", "supports_streaming", "supports_tools",
                    "supports_vision", "is_local")
    _JSONB = ("category_scores", "modalities")

    def upsert_model_ranking(self, model_id, **fields):
        f = {k: v for k, v in fields.items() if k in self._RANK_FIELDS and v is not None}
        cols = ["model_id"] + list(f)
        vals = [model_id] + [f[k] for k in f]
        ph = ", ".join(f"${i + 1}" + ("::jsonb" if c in self._JSONB else "")
                       for i, c in enumerate(cols))
        upd = ", ".join(f"{c} = EXCLUDED.{c}" for c in f)
        self._q(f"INSERT INTO model_rankings ({', '.join(cols)}) VALUES ({ph}) ON CONFLICT "
                f"(model_id) DO UPDATE SET " + (upd + ", " if upd else "") + "updated_at = now()",
                *vals)

    def list_model_rankings(self):
        return self._q("SELECT * FROM model_rankings ORDER BY model_id")

    def update_model_stats(self, model_id, tokens_in, tokens_out, latency_ms, cost, ok):
        self._q("INSERT INTO model_stats (model_id, total_requests, total_tokens_in, "
                "total_tokens_out, total_cost_usd, avg_duration_ms, error_count, last_used_at) "
                "VALUES ($1, 1, $2, $3, $4, $5, $6, now()) ON CONFLICT (model_id) DO UPDATE SET "
                "avg_duration_ms = (model_stats.avg_duration_ms * model_stats.total_requests "
                "  + EXCLUDED.avg_duration_ms) / (model_stats.total_requests + 1), "
                "total_requests = model_stats.total_requests + 1, "
                "total_tokens_in = model_stats.total_tokens_in + EXCLUDED.total_tokens_in, "
                "total_tokens_out = model_stats.total_tokens_out + EXCLUDED.total_tokens_out, "
                "total_cost_usd = model_stats.total_cost_usd + EXCLUDED.total_cost_usd, "
                "error_count = model_stats.error_count + EXCLUDED.error_count, "
                "last_used_at = now(), updated_at = now()",
                model_id, int(tokens_in), int(tokens_out), float(cost), float(latency_ms),
                0 if ok else 1)

    def feedback(self, model_id, good):
        col = "feedback_positive" if good else "feedback_negative"
        self._q(f"INSERT INTO model_stats (model_id, {col}) VALUES ($1, 1) ON CONFLICT "
                f"(model_id) DO UPDATE SET {col} = model_stats.{col} + 1, updated_at = now()",
                model_id)
        return True

    def model_stats(self):
        return self._q("SELECT model_id, total_requests, total_tokens_in::int AS total_tokens_in, "
                       "total_tokens_out::int AS total_tokens_out, "
                       "total_cost_usd::float8 AS total_cost_usd, "
                       "avg_duration_ms::float8 AS avg_duration_ms, error_count, "
                       "feedback_positive, feedback_negative, last_used_at, "
                       "success_rate::float8 AS success_rate, "
                       "avg_cost_per_request::float8 AS avg_cost_per_request FROM model_stats")

    def device_stats_7d(self, device_id):
        r = self._one("SELECT total_jobs_7d::int AS total, done_jobs_7d::int AS done, "
                      "avg_latency_ms::float8 AS ms FROM v_device_stats WHERE device_id = $1",
                      device_id)
        if r is None:
            return {"total_jobs_7d": 0, "done_jobs_7d": 0, "success_rate": 0.0,
                    "avg_latency_ms": 0}
        return {"total_jobs_7d": r["total"], "done_jobs_7d": r["done"],
                "success_rate": (r["done"] / r["total"]) if r["total"] else 0.0,
                "avg_latency_ms": int(r["ms"] or 0)}
