"""Synchronous gRPC client of llmmcp.v1.Core (used by workers, the bridge
and tests).  Mirrors the worker's calls in the reference
(worker/llm_worker/main.py:51-99) plus the lease-token fields."""
from __future__ import annotations

import json

import grpc

from . import proto as pb


class CoreClient:
    def __init__(self, addr: str, timeout: float = 10.0):
        if addr.startswith(":"):
            addr = "127.0.0.1" + addr
        self.channel = grpc.insecure_channel(addr)
        self.timeout = timeout
        self._stubs = {}
        for name, (inp, out, streaming) in pb.METHODS.items():
            path = f"/{pb.SERVICE}/{name}"
            mk = self.channel.unary_stream if streaming else self.channel.unary_unary
            self._stubs[name] = mk(path, request_serializer=pb.msgs[inp].SerializeToString,
                                   response_deserializer=pb.msgs[out].FromString)

    def call(self, name: str, req, timeout: float | None = None, metadata=None):
        return self._stubs[name](req, timeout=timeout or self.timeout, metadata=metadata)

    # convenience ------------------------------------------------------------
    def submit(self, kind, payload=None, priority=0, source="", max_attempts=0, deadline_at="",
               request_id=""):
        """``request_id`` travels as ``x-request-id`` call metadata and is kept
        in the job payload (utils/tracing.py)."""
        md = (("x-request-id", request_id),) if request_id else None
        return self.call("SubmitJob", pb.SubmitJobRequest(
            kind=kind, payload_json=json.dumps(payload or {}), priority=priority, source=source,
            max_attempts=max_attempts, deadline_at=deadline_at), metadata=md).job_id

    def get(self, job_id):
        return job_dict(self.call("GetJob", pb.GetJobRequest(job_id=job_id)).job)

    def stream(self, job_id, timeout=3600):
        for ev in self._stubs["StreamJob"](pb.StreamJobRequest(job_id=job_id), timeout=timeout):
            yield {"job_id": ev.job_id, "type": ev.type, "message": ev.message, "ts": ev.ts,
                   "data": json.loads(ev.data_json or "{}")}

    def register(self, worker_id="", name="", platform="", arch="", host="", tags=None):
        return self.call("RegisterWorker", pb.RegisterWorkerRequest(worker=pb.WorkerInfo(
            id=worker_id, name=name, platform=platform, arch=arch, host=host,
            tags_json=json.dumps(tags or {})))).worker_id

    def claim(self, worker_id, kinds=(), lease_seconds=60, device_id="", wait_ms=0):
        r = self.call("ClaimJob", pb.ClaimJobRequest(worker_id=worker_id, kinds=list(kinds),
                                                     lease_seconds=lease_seconds,
                                                     device_id=device_id, wait_ms=wait_ms),
                      timeout=self.timeout + wait_ms / 1000.0)
        return job_dict(r.job) if r.HasField("job") and r.job.id else None

    def heartbeat(self, worker_id, job_id, extend_seconds=30, attempt_id=""):
        return self.call("Heartbeat", pb.HeartbeatRequest(
            worker_id=worker_id, job_id=job_id, extend_seconds=extend_seconds,
            attempt_id=attempt_id)).ok

    def progress(self, worker_id, job_id, progress: dict, extend_seconds=30, attempt_id=""):
        """Heartbeat carrying a progress report (job SSE ``event: progress``)."""
        return self.call("Heartbeat", pb.HeartbeatRequest(
            worker_id=worker_id, job_id=job_id, extend_seconds=extend_seconds,
            attempt_id=attempt_id, progress_json=json.dumps(progress))).ok

    def complete(self, worker_id, job_id, result, metrics=None, attempt_id=""):
        return self.call("CompleteJob", pb.CompleteJobRequest(
            worker_id=worker_id, job_id=job_id, result_json=json.dumps(result),
            metrics_json=json.dumps(metrics or {}), attempt_id=attempt_id)).ok

    def fail(self, worker_id, job_id, error, metrics=None, attempt_id=""):
        r = self.call("FailJob", pb.FailJobRequest(
            worker_id=worker_id, job_id=job_id, error=error,
            metrics_json=json.dumps(metrics or {}), attempt_id=attempt_id))
        return r.status if r.ok else None

    def report_metrics(self, worker: dict, metrics: dict):
        return self.call("ReportMetrics", pb.ReportMetricsRequest(
            worker=pb.WorkerInfo(id=worker.get("id", ""), name=worker.get("name", ""),
                                 platform=worker.get("platform", ""), arch=worker.get("arch", ""),
                                 host=worker.get("host", ""),
                                 tags_json=json.dumps(worker.get("tags") or {})),
            metrics_json=json.dumps(metrics))).ok

    def report_benchmark(self, device_id, model_id, task_type, tokens_in, tokens_out,
                         latency_ms, tps, meta=None):
        return self.call("ReportBenchmark", pb.ReportBenchmarkRequest(benchmark=pb.Benchmark(
            device_id=device_id, model_id=model_id, task_type=task_type, tokens_in=tokens_in,
            tokens_out=tokens_out, latency_ms=latency_ms, tps=tps,
            meta_json=json.dumps(meta or {})))).ok

    def close(self):
        self.channel.close()


def job_dict(m) -> dict:
    return {"id": m.id, "kind": m.kind, "payload": json.loads(m.payload_json or "{}"),
            "status": m.status, "attempts": m.attempts, "max_attempts": m.max_attempts,
            "lease_until": m.lease_until or None, "deadline_at": m.deadline_at or None,
            "result": json.loads(m.result_json) if m.result_json else None,
            "error": m.error or None, "priority": m.priority, "queued_at": m.queued_at,
            "updated_at": m.updated_at, "attempt_id": m.attempt_id or None}
