"""Claim -> heartbeat -> execute -> complete/fail loop of a GPU worker
(reference: worker/llm_worker/main.py:536-599).

Differences, MI355X-first:
  * concurrency: a GPU worker keeps up to ``capacity`` jobs in flight, all fed
    to the same continuous-batching engine (the reference ran one job at a time
    per worker process);
  * wake-up: long-poll claims (``wait_ms``) instead of a 1.5 s idle sleep;
  * every call carries the lease token, so a worker whose lease expired cannot
    overwrite the new owner's result;
  * heartbeat every max(5, lease/2) s per in-flight job; while a job reports
    progress (tokens generated so far) a changed report rides on a heartbeat
    every ``progress_s`` (job SSE ``event: progress``);
  * a GPU/engine failure fails the job (requeued by attempts) and reports the
    device offline so discovery/routing stop sending it work;
  * admission by KV capacity, not a fixed DEVICE_MAX_CONCURRENCY (SURVEY
    §7.5 item 4): while the engine's queue is backed up or its paged KV cache
    is nearly full the agent stops claiming, so queued jobs stay in the shared
    queue for a less loaded GPU instead of waiting behind this one.
"""
from __future__ import annotations

import asyncio
import logging
import os
import socket
import time

from ..store.base import parse_iso
from ..utils import tracing
from ..utils.faults import faults
from .jobs import JobError, JobRunner

log = logging.getLogger("lmx.worker")

NETWORK_TOKENS = ("connection refused", "timed out", "timeout", "no route",
                  "network is unreachable")


def should_mark_offline(exc: Exception) -> bool:
    msg = str(exc).lower()
    if "hip" in msg or "cuda" in msg or "device" in msg and "error" in msg:
        return True
    return any(t in msg for t in NETWORK_TOKENS)


class WorkerAgent:
    def __init__(self, client, runner: JobRunner, device_id: str, worker_id: str = "",
                 kinds: list[str] | None = None, lease_s: int = 60, capacity: int = 64,
                 name: str = "", tags: dict | None = None, mark_offline=None,
                 health=None, admit=None, progress_s: float | None = None):
        self.client = client  # rpc.client.CoreClient (sync; called via to_thread)
        self.runner = runner
        self.device_id = device_id
        self.worker_id = worker_id
        self.kinds = list(kinds or [])
        self.lease_s = lease_s
        self.capacity = capacity
        self.name = name or socket.gethostname()
        self.tags = dict(tags or {})
        self.mark_offline = mark_offline  # callable(device_id, reason) or None
        # callable() -> (ok, reason): a hung or failed engine stops heartbeating
        # so the core requeues its leases when they expire
        self.health = health
        self._reported_unhealthy = False
        # callable() -> (ok, reason): engine-side admission (KV pages, backlog)
        self.admit = admit
        # progress report cadence (s); a report is sent only when it changed
        self.progress_s = progress_s if progress_s is not None else \
            float(os.environ.get("LMX_PROGRESS_S", "2"))
        self.inflight: dict[str, asyncio.Task] = {}
        self._stop = asyncio.Event()
        self.stats = {"claimed": 0, "done": 0, "failed": 0, "lease_lost": 0}

    async def register(self, retry_s: float = 2.0):
        while not self._stop.is_set():
            try:
                self.worker_id = await asyncio.to_thread(
                    self.client.register, self.worker_id, self.name, "rocm", "gfx950",
                    socket.gethostname(), {**self.tags, "device_id": self.device_id})
                log.info("registered as %s", self.worker_id)
                return self.worker_id
            except Exception as e:
                log.warning("register failed: %s", e)
                await asyncio.sleep(retry_s)

    def stop(self):
        self._stop.set()

    async def run(self, max_jobs: int | None = None):
        # always (re-)register: a preset worker id must still appear in the
        # devices table (dashboard workers_online, capacity, telemetry)
        await self.register()
        n = 0
        while not self._stop.is_set():
            if len(self.inflight) >= self.capacity:
                await asyncio.wait(list(self.inflight.values()),
                                   return_when=asyncio.FIRST_COMPLETED)
                continue
            if self.health is not None:
                ok, why = self.health()
                if not ok:
                    # a broken GPU pulls no new work: the queue hands it to the
                    # healthy devices (the worker process exits and is restarted)
                    self.stats["unhealthy_waits"] = self.stats.get("unhealthy_waits", 0) + 1
                    await asyncio.sleep(0.2)
                    continue
            if self.admit is not None and self.inflight:
                ok, _why = self.admit()
                if not ok:
                    self.stats["admission_waits"] = self.stats.get("admission_waits", 0) + 1
                    await asyncio.wait(list(self.inflight.values()), timeout=0.05,
                                       return_when=asyncio.FIRST_COMPLETED)
                    continue
            try:
                j = await asyncio.to_thread(self.client.claim, self.worker_id, self.kinds,
                                            self.lease_s, self.device_id, 2000)
            except Exception as e:
                log.warning("claim failed: %s", e)
                await asyncio.sleep(1.0)
                continue
            if j is None:
                continue
            self.stats["claimed"] += 1
            if faults().hit("claim_drop"):     # vanish with the lease: it must expire
                self.stats["dropped"] = self.stats.get("dropped", 0) + 1
                continue
            t = asyncio.create_task(self._run_job(j))
            self.inflight[j["id"]] = t
            t.add_done_callback(lambda _t, jid=j["id"]: self.inflight.pop(jid, None))
            n += 1
            if max_jobs is not None and n >= max_jobs:
                break
        if self.inflight:
            await asyncio.gather(*self.inflight.values(), return_exceptions=True)

    async def _heartbeat(self, jid: str, token: str, prog: dict | None = None):
        """Lease extension every max(5, lease/2) s.  While the job updates
        ``prog`` (tokens so far) a changed report is sent every ``progress_s``
        instead, as a heartbeat carrying it (job SSE ``event: progress``)."""
        period = max(5.0, self.lease_s / 2)
        send_prog = getattr(self.client, "progress", None) if prog is not None else None
        tick = min(period, self.progress_s) if send_prog is not None else period
        last_ext, sent = time.monotonic(), None
        while True:
            await asyncio.sleep(tick)
            changed = send_prog is not None and bool(prog) and prog != sent
            if not changed and time.monotonic() - last_ext < period - 1e-3:
                continue
            if self.health is not None:
                ok, why = self.health()
                if not ok:
                    # let the lease lapse: the core hands the job to another GPU
                    log.error("engine unhealthy (%s): not extending %s", why, jid)
                    if not self._reported_unhealthy and self.mark_offline:
                        self._reported_unhealthy = True
                        try:
                            await asyncio.to_thread(self.mark_offline, self.device_id, why)
                        except Exception:
                            pass
                    continue
            try:
                if changed:
                    snap = dict(prog)
                    ok = await asyncio.to_thread(send_prog, self.worker_id, jid, snap,
                                                 self.lease_s, token)
                    sent = snap
                    self.stats["progress_sent"] = self.stats.get("progress_sent", 0) + 1
                else:
                    ok = await asyncio.to_thread(self.client.heartbeat, self.worker_id, jid,
                                                 self.lease_s, token)
                last_ext = time.monotonic()
                if not ok:
                    log.warning("lease lost for %s", jid)
                    self.stats["lease_lost"] += 1
                    return
            except Exception as e:
                log.warning("heartbeat %s failed: %s", jid, e)

    async def _run_job(self, j: dict):
        jid, token = j["id"], j.get("attempt_id") or ""
        prog: dict = {}
        hb = asyncio.create_task(self._heartbeat(jid, token, prog))
        t0 = time.time()
        # correlation: the submitter's X-Request-ID if it rode in the payload,
        # else the job id (utils/tracing.py)
        rid = tracing.payload_request_id(j.get("payload")) or jid
        q = j.get("queued_at")
        try:   # ISO string (HTTP / gRPC) or epoch seconds (in-process store)
            queued = float(q) if isinstance(q, (int, float)) else parse_iso(q)
        except (TypeError, ValueError, AttributeError):
            queued = None
        span = {"job_id": jid, "kind": j.get("kind", ""), "device_id": self.device_id,
                "attempt": j.get("attempts"),
                "queue_wait_ms": None if queued is None else max(0.0, t0 - queued) * 1e3}
        try:
            faults().maybe_raise("job_crash", "injected job crash")
            result, metrics = await self.runner.handle(j["kind"], j.get("payload") or {},
                                                       progress=prog)
            metrics = dict(metrics or {})
            metrics.setdefault("ms", int((time.time() - t0) * 1000))
            metrics.setdefault("request_id", rid)
            ok = await asyncio.to_thread(self.client.complete, self.worker_id, jid, result,
                                         metrics, token)
            self.stats["done" if ok else "lease_lost"] += 1
            tracing.record_span("job.attempt", rid, status="done" if ok else "lease_lost",
                                run_ms=(time.time() - t0) * 1e3, ttft_ms=prog.get("ttft_ms"),
                                tokens_in=prog.get("tokens_in"),
                                tokens_out=prog.get("tokens_out"), **span)
        except Exception as e:
            self.stats["failed"] += 1
            log.warning("job %s failed: %s", jid, e)
            tracing.record_span("job.attempt", rid, status="failed", error=str(e)[:200],
                                run_ms=(time.time() - t0) * 1e3, **span)
            try:
                await asyncio.to_thread(self.client.fail, self.worker_id, jid, str(e),
                                        {"ms": int((time.time() - t0) * 1000)}, token)
            except Exception as e2:
                log.warning("fail report for %s failed: %s", jid, e2)
            if not isinstance(e, JobError) and should_mark_offline(e) and self.mark_offline:
                try:
                    await asyncio.to_thread(self.mark_offline, self.device_id, str(e))
                except Exception:
                    pass
        finally:
            hb.cancel()


def engine_admission(engine, max_waiting: int | None = None, kv_high: float = 0.92):
    """Admission predicate for a chat engine: claim more work only while the
    engine's waiting queue is short and its KV cache has headroom."""
    limit = max_waiting if max_waiting is not None else max(4, engine.ecfg.max_num_seqs // 4)

    def admit():
        s = engine.sched
        if s.num_waiting >= limit:
            return False, f"engine backlog {s.num_waiting}"
        if s.kv_usage >= kv_high:
            return False, f"kv cache {s.kv_usage:.0%} full"
        return True, ""
    return admit
