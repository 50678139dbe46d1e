"""gRPC server for llmmcp.v1.Core (reference: core/internal/grpcserver/server.go).

Runs on the core's asyncio loop (grpc.aio) next to the HTTP server.  Fixes of
the reference's gRPC-path defects:
  * ClaimJob enforces per-device concurrency and device-online like the HTTP
    claim (the reference's gRPC claim did not), and can long-poll (wait_ms);
  * CompleteJob / FailJob record cost and feed the circuit breaker;
  * StreamJob wakes on store change notifications instead of a 1 s poll;
  * lease tokens (attempt_id) are honoured on heartbeat / complete / fail.
Invalid JSON in *_json fields is replaced by {} (sanitizeJSON, server.go:400).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time

import grpc

from ..store.base import iso, parse_iso
from ..utils import tracing
from . import proto as pb

log = logging.getLogger("lmx.grpc")


def sanitize_json(s: str, default=None):
    if default is None:
        default = {}
    if not s or not s.strip():
        return default
    try:
        return json.loads(s)
    except ValueError:
        return default


def job_msg(j: dict):
    return pb.Job(id=j["id"], kind=j["kind"], payload_json=json.dumps(j.get("payload") or {}),
                  status=j["status"], attempts=j["attempts"], max_attempts=j["max_attempts"],
                  lease_until=iso(j.get("lease_until")) or "",
                  deadline_at=iso(j.get("deadline_at")) or "",
                  result_json=json.dumps(j["result"]) if j.get("result") is not None else "",
                  error=j.get("error") or "", priority=j.get("priority", 0),
                  queued_at=iso(j.get("queued_at")) or "", updated_at=iso(j.get("updated_at")) or "",
                  attempt_id=j.get("attempt_id") or "")


class CoreService:
    def __init__(self, state):
        self.st = state

    @property
    def store(self):
        return self.st.store

    async def _db(self, fn, *a):
        if getattr(self.store, "backend", "memory") == "memory":
            return fn(*a)
        return await asyncio.to_thread(fn, *a)

    async def SubmitJob(self, req, ctx):
        if not req.kind.strip():
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "kind_required")
        deadline = None
        if req.deadline_at:
            try:
                deadline = parse_iso(req.deadline_at)
            except ValueError:
                await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "invalid_deadline_at")
        payload = sanitize_json(req.payload_json)
        if isinstance(payload, dict):
            # request id from the call metadata (utils/tracing.py), as X-Request-ID over HTTP
            rid = ""
            for item in ctx.invocation_metadata() or ():
                k, v = item if isinstance(item, tuple) else (item.key, item.value)
                if k == "x-request-id":
                    rid = tracing.clean_id(v)
            payload = tracing.tag_payload(payload, rid)
        jid = await self._db(self.store.submit_job, req.kind, payload,
                             req.priority, req.source, req.max_attempts or 3, deadline)
        self.st.metrics.jobs_created.labels(req.kind).inc()
        return pb.SubmitJobResponse(job_id=jid)

    async def GetJob(self, req, ctx):
        j = await self._db(self.store.get_job, req.job_id)
        if j is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, "not_found")
        return pb.GetJobResponse(job=job_msg(j))

    async def StreamJob(self, req, ctx):
        j = await self._db(self.store.get_job, req.job_id)
        if j is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, "not_found")
        last = None
        ver = self.store.job_version()
        while True:
            if j["status"] != last:
                last = j["status"]
                yield pb.JobEvent(job_id=j["id"], type="status", message=j["status"],
                                  ts=iso(time.time()),
                                  data_json=json.dumps({"status": j["status"],
                                                        "result": j.get("result"),
                                                        "error": j.get("error")}))
            if j["status"] in ("done", "error"):
                return
            ver = await self.st.job_hub().wait(ver, 15.0)
            j = await self._db(self.store.get_job, req.job_id)
            if j is None:
                return

    async def RegisterWorker(self, req, ctx):
        w = req.worker
        wid = w.id.strip() or f"worker-{time.time_ns()}"
        tags = sanitize_json(w.tags_json)
        await self._db(self.store.upsert_device, wid, w.name, w.platform, w.arch, w.host,
                       tags, "online")
        from ..api.routes import revive_engine_device
        await self._db(revive_engine_device, self.store,
                       tags if isinstance(tags, dict) else {})
        return pb.RegisterWorkerResponse(worker_id=wid)

    async def ClaimJob(self, req, ctx):
        if not req.worker_id.strip():
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "worker_id_required")
        j = await self.st.control._claim(req.worker_id, list(req.kinds),
                                         req.lease_seconds or 60, req.device_id,
                                         min(req.wait_ms, 30000))
        return pb.ClaimJobResponse(job=job_msg(j)) if j else pb.ClaimJobResponse()

    async def Heartbeat(self, req, ctx):
        prog = sanitize_json(req.progress_json) if req.progress_json else None
        ok = await self._db(self.store.heartbeat, req.job_id, req.worker_id,
                            req.extend_seconds or 30, req.attempt_id, prog)
        return pb.HeartbeatResponse(ok=bool(ok))

    async def CompleteJob(self, req, ctx):
        metrics = sanitize_json(req.metrics_json)
        result = sanitize_json(req.result_json)
        ok = await self._db(self.store.complete_job, req.job_id, req.worker_id, result, metrics,
                            req.attempt_id)
        if ok:
            await self._db(self.st.control._record_cost, req.job_id,
                           metrics if isinstance(metrics, dict) else {})
            j = await self._db(self.store.get_job, req.job_id) or {}
            dev = (result.get("device_id") if isinstance(result, dict) else None) or \
                j.get("device_id")
            if dev:
                self.st.circuit.record(dev, True)
        return pb.CompleteJobResponse(ok=bool(ok))

    async def FailJob(self, req, ctx):
        j = await self._db(self.store.get_job, req.job_id)
        if j is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, "not_found")
        st = await self._db(self.store.fail_job, req.job_id, req.worker_id, req.error,
                            sanitize_json(req.metrics_json), req.attempt_id)
        if st is not None:
            dev = j.get("device_id") or (j.get("payload") or {}).get("device_id")
            if dev:
                self.st.circuit.record(dev, False)
        return pb.FailJobResponse(ok=st is not None, status=st or "")

    async def ReportMetrics(self, req, ctx):
        w = req.worker
        if w.id:
            await self._db(self.store.upsert_device, w.id, w.name, w.platform, w.arch, w.host,
                           sanitize_json(w.tags_json), "online", True)
            await self._db(self.store.insert_device_metrics, w.id, sanitize_json(req.metrics_json))
        return pb.ReportMetricsResponse(ok=True)

    async def ReportBenchmark(self, req, ctx):
        b = req.benchmark
        if b.model_id and not self.store.get_model(b.model_id):
            await self._db(lambda: self.store.upsert_model(b.model_id, provider="local",
                                                            kind="bench"))
        await self._db(self.store.insert_benchmark, b.device_id, b.model_id, b.task_type,
                       b.tokens_in, b.tokens_out, b.latency_ms, b.tps, sanitize_json(b.meta_json))
        return pb.ReportBenchmarkResponse(ok=True)


def generic_handler(service: CoreService):
    handlers = {}
    for name, (inp, out, streaming) in pb.METHODS.items():
        fn = getattr(service, name)
        de = pb.msgs[inp].FromString
        se = pb.msgs[out].SerializeToString
        if streaming:
            handlers[name] = grpc.unary_stream_rpc_method_handler(
                fn, request_deserializer=de, response_serializer=se)
        else:
            handlers[name] = grpc.unary_unary_rpc_method_handler(
                fn, request_deserializer=de, response_serializer=se)
    return grpc.method_handlers_generic_handler(pb.SERVICE, handlers)


def reflection_handler():
    """grpc.reflection.v1alpha.ServerReflection (and the v1 name) over the
    runtime-built descriptors, so grpcurl / grpc_cli can list and describe
    llmmcp.v1.Core.  The reference documents reflection but never registers
    it (doc/README.md:352-357 vs core/cmd/core/main.go:92-93)."""
    R = pb.reflection
    services = [pb.SERVICE, pb.REFLECTION_SERVICE]
    files = {pb.FILE.name: pb.FILE, pb.REFLECTION_FILE.name: pb.REFLECTION_FILE}

    def file_for_symbol(sym: str):
        for f in files.values():
            if sym == f.package or sym.startswith(f.package + "."):
                return f
        return None

    async def info(request_iterator, context):
        async for req in request_iterator:
            resp = R["ServerReflectionResponse"](valid_host=req.host, original_request=req)
            f = None
            if req.list_services:
                resp.list_services_response.service.extend(
                    [R["ServiceResponse"](name=n) for n in services])
            elif req.file_by_filename or req.file_containing_symbol:
                f = files.get(req.file_by_filename) if req.file_by_filename else \
                    file_for_symbol(req.file_containing_symbol)
                if f is None:
                    resp.error_response.error_code = grpc.StatusCode.NOT_FOUND.value[0]
                    resp.error_response.error_message = "symbol or file not found"
                else:
                    resp.file_descriptor_response.file_descriptor_proto.append(
                        f.SerializeToString())
            else:
                resp.error_response.error_code = grpc.StatusCode.UNIMPLEMENTED.value[0]
                resp.error_response.error_message = "request kind not supported"
            yield resp

    h = grpc.stream_stream_rpc_method_handler(
        info, request_deserializer=R["ServerReflectionRequest"].FromString,
        response_serializer=R["ServerReflectionResponse"].SerializeToString)
    return [grpc.method_handlers_generic_handler(pb.REFLECTION_SERVICE,
                                                 {"ServerReflectionInfo": h}),
            grpc.method_handlers_generic_handler("grpc.reflection.v1.ServerReflection",
                                                 {"ServerReflectionInfo": h})]


async def start_grpc(state, addr: str | None = None):
    addr = addr or os.environ.get("CORE_GRPC_ADDR", ":9090")
    if addr.startswith(":"):
        addr = "0.0.0.0" + addr
    server = grpc.aio.server()
    server.add_generic_rpc_handlers((generic_handler(CoreService(state)),
                                     *reflection_handler()))
    port = server.add_insecure_port(addr)
    await server.start()
    log.info("gRPC listening on %s", addr)
    return server, port
