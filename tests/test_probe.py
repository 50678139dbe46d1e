"""Probe harness (C19, reference scripts/probe_openrouter_models.py) against the
in-process core app with a scripted worker completing the probe jobs."""
import asyncio
from aiohttp.test_utils import TestClient, TestServer

from llm_mcp_amd.api.core import CoreState, create_core_app
from llm_mcp_amd.bench import probe
from llm_mcp_amd.store.memory import MemoryStore


def _args(base, **kw):
    a = probe.parser().parse_args(["--base-url", base, "--models", "llama-3-8b",
                                   "--runs-per-model", "3", "--poll-sec", "0.02",
                                   "--job-timeout-sec", "10"])
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_usage_fallbacks():
    assert probe.usage({"tokens_in": 5, "tokens_out": 7}, "x" * 40) == (5, 7)
    assert probe.usage({"response": "y" * 40}, "x" * 40) == (10, 10)
    assert probe.usage({"data": {"choices": [{"message": {"content": "z" * 8}}]}}, "") == (1, 2)


def test_probe_through_job_queue(monkeypatch):
    monkeypatch.setenv("LMX_FAKE_GPUS", "1:288")
    monkeypatch.setenv("LMX_NODE_ID", "node1")
    monkeypatch.delenv("LMX_ALLOW_CLOUD", raising=False)

    async def go():
        st = CoreState(store=MemoryStore())
        c = TestClient(TestServer(create_core_app(st, background=False)))
        async with c:
            base = str(c.make_url("")).rstrip("/")
            stop = asyncio.Event()

            async def worker():
                n = 0
                while not stop.is_set():
                    r = await (await c.post("/v1/workers/claim",
                                            json={"worker_id": "wp"})).json()
                    job = r.get("job")
                    if not job:
                        await asyncio.sleep(0.01)
                        continue
                    n += 1
                    if n == 2:      # one failing attempt: requeued, retried
                        await c.post("/v1/workers/fail", json={
                            "worker_id": "wp", "job_id": job["id"], "error": "boom",
                            "attempt_id": job["attempt_id"]})
                        continue
                    await c.post("/v1/workers/complete", json={
                        "worker_id": "wp", "job_id": job["id"], "attempt_id": job["attempt_id"],
                        "result": {"ok": True, "response": "w" * 64, "tokens_in": 12,
                                   "tokens_out": 16, "device_id": "node1-gpu0"}})

            wt = asyncio.create_task(worker())
            try:
                runs, summary = await probe.run_probe(_args(base))
            finally:
                stop.set()
                await wt
            return runs, summary

    runs, summary = asyncio.new_event_loop().run_until_complete(go())
    assert [r.ok for r in runs] == [True, True, True]
    assert all(r.tokens_out == 16 and r.device_id == "node1-gpu0" for r in runs)
    assert any(r.meta["attempts"] == 2 for r in runs)
    s = summary["llama-3-8b"]
    assert s["ok"] == 3 and s["latency_p95_ms"] >= s["latency_p50_ms"] > 0
    rows = []
    assert probe.record(runs, lambda *a: rows.append(a)) == 3
    assert rows[0][:3] == ("node1-gpu0", "llama-3-8b", "probe.generate")


def test_rejected_request_is_reported():
    async def go():
        st = CoreState(store=MemoryStore())
        c = TestClient(TestServer(create_core_app(st, background=False)))
        async with c:
            base = str(c.make_url("")).rstrip("/")
            a = _args(base, quality="bogus")
            import aiohttp
            async with aiohttp.ClientSession() as s:
                return await probe.probe_one(s, base, "", 0, a)

    pr = asyncio.new_event_loop().run_until_complete(go())
    assert pr.status == "rejected" and not pr.ok and pr.error
