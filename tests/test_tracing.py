"""Request-ID propagation and per-request spans: HTTP header in
and out, job payload tagging, worker attempt span, /v1/debug/trace."""
import asyncio

from aiohttp.test_utils import TestClient, TestServer

from llm_mcp_amd.api.core import CoreState, create_core_app
from llm_mcp_amd.store.memory import MemoryStore
from llm_mcp_amd.utils import tracing


def run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def test_clean_and_tag():
    assert tracing.clean_id("abc-123") == "abc-123"
    assert tracing.clean_id("x" * 200) == ""
    assert tracing.clean_id("bad\nid") == ""
    assert tracing.clean_id(None) == ""
    p = {"a": 1}
    assert tracing.tag_payload(p, "") is p
    q = tracing.tag_payload(p, "r1")
    assert q == {"a": 1, "_request_id": "r1"} and p == {"a": 1}
    # an ID already in the payload wins
    assert tracing.tag_payload(q, "r2")["_request_id"] == "r1"
    assert tracing.payload_request_id(q) == "r1"
    assert tracing.payload_request_id("nope") == ""


def test_span_ring_bounded_and_searchable():
    ring = tracing.SpanRing(maxlen=3)
    for i in range(5):
        ring.add({"request_id": f"r{i % 2}", "i": i})
    assert [s["i"] for s in ring.find("r0")] == [2, 4]
    assert [s["i"] for s in ring.find("r1")] == [3]


def test_http_request_id_roundtrip_and_job_tagging(monkeypatch):
    monkeypatch.setenv("LMX_FAKE_GPUS", "1:288")
    monkeypatch.setenv("LMX_NODE_ID", "node1")

    async def go():
        st = CoreState(store=MemoryStore())
        c = TestClient(TestServer(create_core_app(st, background=False)))
        async with c:
            r = await c.get("/health")
            minted = r.headers.get("X-Request-ID")
            assert minted and len(minted) == 32
            r = await c.get("/health", headers={"X-Request-ID": "trace-42"})
            assert r.headers["X-Request-ID"] == "trace-42"
            # error responses carry it too
            r = await c.get("/v1/jobs", headers={"X-Request-ID": "trace-43"})
            assert r.status == 405 and r.headers["X-Request-ID"] == "trace-43"
            # a client ID is carried into the job payload ...
            r = await c.post("/v1/jobs", json={"kind": "echo", "payload": {"x": 1}},
                             headers={"X-Request-ID": "trace-44"})
            jid = (await r.json())["job_id"]
            j = await (await c.get(f"/v1/jobs/{jid}")).json()
            assert j["payload"] == {"x": 1, "_request_id": "trace-44"}
            # ... a minted one is not (payload stays as submitted)
            r = await c.post("/v1/jobs", json={"kind": "echo", "payload": {"y": 2}})
            jid2 = (await r.json())["job_id"]
            j = await (await c.get(f"/v1/jobs/{jid2}")).json()
            assert j["payload"] == {"y": 2}
            r = await c.get("/v1/debug/trace/never-seen")
            assert r.status == 404
            tracing.record_span("unit", "trace-45", a=1.23456)
            r = await c.get("/v1/debug/trace/trace-45")
            body = await r.json()
            assert r.status == 200 and body["spans"][0]["a"] == 1.235
    run(go())


class _Client:
    """In-memory stand-in for the core client used by WorkerAgent."""

    def __init__(self):
        self.completed = []

    def complete(self, worker_id, jid, result, metrics, token):
        self.completed.append((jid, result, metrics))
        return True

    def fail(self, *a):
        return True

    def heartbeat(self, *a):
        return True


class _Runner:
    async def handle(self, kind, payload, progress=None):
        if progress is not None:
            progress.update(tokens_in=3, tokens_out=5, ttft_ms=7)
        if kind == "boom":
            raise RuntimeError("kaput")
        return {"ok": True}, {"ms": 1}


def test_worker_attempt_span():
    from llm_mcp_amd.store.base import iso
    from llm_mcp_amd.worker.agent import WorkerAgent
    import time

    cl = _Client()
    ag = WorkerAgent(cl, _Runner(), "gpu0", worker_id="w1", lease_s=60)
    job = {"id": "job-1", "kind": "engine.generate", "attempts": 1, "attempt_id": "tok",
           "queued_at": iso(time.time() - 2.0), "payload": {"_request_id": "trace-w1"}}
    run(ag._run_job(job))
    assert cl.completed[0][2]["request_id"] == "trace-w1"
    sp = tracing.RING.find("trace-w1")[-1]
    assert sp["span"] == "job.attempt" and sp["status"] == "done" and sp["job_id"] == "job-1"
    assert sp["tokens_out"] == 5 and sp["ttft_ms"] == 7 and sp["queue_wait_ms"] >= 1900
    # no request id in the payload: the job id is the correlation key
    run(ag._run_job({"id": "job-2", "kind": "boom", "payload": {}}))
    sp = tracing.RING.find("job-2")[-1]
    assert sp["status"] == "failed" and "kaput" in sp["error"]
