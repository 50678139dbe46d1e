"""HTTP control plane against the memory store (reference contracts:
core/internal/api/handlers.go)."""
import asyncio
import json
import time

import pytest
from aiohttp.test_utils import TestClient, TestServer

from llm_mcp_amd.api.core import CoreState, create_core_app
from llm_mcp_amd.store.memory import MemoryStore


@pytest.fixture(autouse=True)
def _env(monkeypatch):
    monkeypatch.setenv("LMX_FAKE_GPUS", "2:288")
    monkeypatch.setenv("LMX_NODE_ID", "node1")
    monkeypatch.delenv("LMX_ALLOW_CLOUD", raising=False)
    monkeypatch.setenv("DEVICE_MAX_CONCURRENCY", "1")


def run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def client(state=None):
    st = state or CoreState(store=MemoryStore())
    return st, TestClient(TestServer(create_core_app(st, background=False)))


def test_health_version_metrics_405():
    async def go():
        st, c = client()
        async with c:
            assert (await (await c.get("/health")).json())["status"] == "ok"
            assert "version" in await (await c.get("/version")).json()
            r = await c.get("/v1/jobs")
            assert r.status == 405 and (await r.json())["error"] == "method_not_allowed"
            assert "llmcore_jobs_created_total" in await (await c.get("/metrics")).text()
    run(go())


def test_job_lifecycle_with_lease_tokens():
    async def go():
        st, c = client()
        async with c:
            r = await c.post("/v1/jobs", json={"kind": "echo", "payload": {"x": 1}})
            assert r.status == 202
            jid = (await r.json())["job_id"]
            j = await (await c.get(f"/v1/jobs/{jid}")).json()
            assert j["status"] == "queued" and j["payload"] == {"x": 1} and j["max_attempts"] == 3
            assert (await c.get("/v1/jobs/not-a-uuid")).status == 404
            r = await c.post("/v1/jobs", json={"payload": {}})
            assert (await r.json())["error"] == "kind_required"
            r = await c.post("/v1/jobs", data="{bad")
            assert (await r.json())["error"] == "invalid_json"
            r = await c.post("/v1/jobs", json={"kind": "x", "deadline_at": "tomorrow"})
            assert (await r.json())["error"] == "invalid_deadline_at"
            w = (await (await c.post("/v1/workers/register",
                                     json={"worker": {"name": "w"}})).json())["worker_id"]
            assert w.startswith("worker-")
            r = await (await c.post("/v1/workers/claim", json={"worker_id": w,
                                                               "lease_seconds": 30})).json()
            job = r["job"]
            assert job["id"] == jid and job["status"] == "running" and job["attempts"] == 1
            tok = job["attempt_id"]
            assert (await (await c.post("/v1/workers/claim", json={"worker_id": w})).json()) == {}
            r = await c.post("/v1/workers/heartbeat", json={"worker_id": w, "job_id": jid,
                                                            "attempt_id": tok})
            assert (await r.json())["ok"] is True
            # a stale token cannot complete the job
            r = await c.post("/v1/workers/complete", json={"worker_id": w, "job_id": jid,
                                                           "attempt_id": "bogus", "result": {}})
            assert r.status == 409
            r = await c.post("/v1/workers/complete", json={
                "worker_id": w, "job_id": jid, "attempt_id": tok, "result": {"ok": True},
                "metrics": {"tokens_in": 3, "tokens_out": 5, "provider": "local",
                            "model": "m"}})
            assert (await r.json())["ok"] is True
            j = await (await c.get(f"/v1/jobs/{jid}")).json()
            assert j["status"] == "done" and j["result"] == {"ok": True}
            assert "lease_until" not in j
            at = await (await c.get(f"/v1/jobs/{jid}/attempts")).json()
            assert at["items"][0]["status"] == "done"
    run(go())


def test_fail_requeues_then_errors():
    async def go():
        st, c = client()
        async with c:
            jid = (await (await c.post("/v1/jobs", json={"kind": "k", "max_attempts": 2})).json())["job_id"]
            for expect in ("queued", "error"):
                job = (await (await c.post("/v1/workers/claim", json={"worker_id": "w1"})).json())["job"]
                r = await c.post("/v1/workers/fail", json={"worker_id": "w1", "job_id": jid,
                                                           "error": "boom",
                                                           "attempt_id": job["attempt_id"]})
                assert (await r.json())["status"] == expect
            j = await (await c.get(f"/v1/jobs/{jid}")).json()
            assert j["status"] == "error" and j["error"] == "boom" and j["attempts"] == 2
            r = await c.post("/v1/workers/fail", json={"worker_id": "w1", "job_id":
                                                       "00000000-0000-4000-8000-000000000000"})
            assert r.status == 404
    run(go())


def test_job_stream_sse():
    async def go():
        st, c = client()
        async with c:
            jid = (await (await c.post("/v1/jobs", json={"kind": "k"})).json())["job_id"]
            resp = await c.get(f"/v1/jobs/{jid}/stream")

            async def worker():
                await asyncio.sleep(0.1)
                j = st.store.claim_job("w", [], 30)
                await asyncio.sleep(0.1)
                st.store.complete_job(jid, "w", {"r": 1}, {}, j["attempt_id"])

            t = asyncio.create_task(worker())
            body = (await resp.read()).decode()
            await t
            events = [json.loads(l[6:]) for l in body.split("\n") if l.startswith("data: ")]
            assert [e["status"] for e in events] == ["queued", "running", "done"]
            assert body.startswith("event: status\n")
    run(go())


def test_job_stream_progress_events():
    """Worker progress reports (heartbeat ``progress``) reach job SSE clients
    as ``event: progress`` frames and GET /v1/jobs/{id} while running."""
    async def go():
        st, c = client()
        async with c:
            jid = (await (await c.post("/v1/jobs", json={"kind": "k"})).json())["job_id"]
            resp = await c.get(f"/v1/jobs/{jid}/stream")
            seen = {}

            async def worker():
                await asyncio.sleep(0.1)
                j = st.store.claim_job("w", [], 30)
                for n in (1, 5):
                    await asyncio.sleep(0.1)
                    r = await c.post("/v1/workers/heartbeat", json={
                        "worker_id": "w", "job_id": jid, "attempt_id": j["attempt_id"],
                        "progress": {"tokens_out": n}})
                    assert (await r.json())["ok"] is True
                seen["running"] = await (await c.get(f"/v1/jobs/{jid}")).json()
                # a stale lease token cannot publish progress
                r = await c.post("/v1/workers/heartbeat", json={
                    "worker_id": "w", "job_id": jid, "attempt_id": "bogus",
                    "progress": {"tokens_out": 99}})
                assert (await r.json())["ok"] is False
                await asyncio.sleep(0.1)
                st.store.complete_job(jid, "w", {"r": 1}, {}, j["attempt_id"])

            t = asyncio.create_task(worker())
            body = (await resp.read()).decode()
            await t
            frames = [f for f in body.split("\n\n") if f.strip()]
            kinds = [f.split("\n")[0][len("event: "):] for f in frames]
            data = [json.loads(f.split("\n")[1][len("data: "):]) for f in frames]
            prog = [d["progress"]["tokens_out"] for k, d in zip(kinds, data) if k == "progress"]
            assert prog == [1, 5]
            assert [d["status"] for k, d in zip(kinds, data) if k == "status"] == \
                ["queued", "running", "done"]
            assert seen["running"]["progress"] == {"tokens_out": 5}
            done = await (await c.get(f"/v1/jobs/{jid}")).json()
            assert done["status"] == "done" and "progress" not in done
    run(go())


def test_discovery_devices_dashboard_capacity():
    async def go():
        st, c = client()
        async with c:
            assert (await c.post("/v1/discovery/run")).status == 200
            last = await (await c.get("/v1/discovery/last")).json()
            assert last["last_run"]
            devs = st.store.list_devices()
            ids = sorted(d["id"] for d in devs)
            assert ids == ["node1:gpu0", "node1:gpu1"]
            assert devs[0]["tags"]["hbm_gb"] == 288 and devs[0]["tags"]["gfx"] == "gfx950"
            d = await (await c.get("/v1/dashboard")).json()
            for k in ("jobs", "benchmarks", "running_jobs", "devices", "hosts", "workers_online",
                      "issues", "costs", "models_count", "updated_at"):
                assert k in d
            assert d["hosts"][0]["id"] == "node1" and len(d["hosts"][0]["nodes"]) == 2
            cap = await (await c.get("/v1/debug/capacity")).json()
            assert cap["total_slots"] == 2
            h = await (await c.get("/v1/debug/health")).json()
            assert set(h["checks"]) >= {"database", "queue", "hosts", "workers"}
            acts = await (await c.get("/v1/debug/actions")).json()
            assert acts["total"] == len(acts["endpoints"]) >= 24
            t = await (await c.post("/v1/debug/test")).json()
            assert [r["name"] for r in t["results"]] == ["db_ping", "db_read", "engine_ping",
                                                         "job_create"]
            # offline device releases its running leases immediately
            jid = st.store.submit_job("k", {"device_id": "node1:gpu0"})
            j = st.store.claim_job("w", [], 60, "node1:gpu0")
            assert j["id"] == jid
            await c.post("/v1/devices/offline", json={"device_id": "node1:gpu0", "reason": "x"})
            assert st.store.get_device("node1:gpu0")["status"] == "offline"
            assert st.store.get_job(jid)["lease_until"] is None
            # the offline report fed the breaker once per released lease (>= 1);
            # three jobs lost on one device trip it (config 5's fault path)
            assert st.circuit.snapshot()["node1:gpu0"]["failures"] == 1
            for _ in range(3):
                st.store.submit_job("k", {"device_id": "node1:gpu1"})
                assert st.store.claim_job("w", [], 60, "node1:gpu1", 8) is not None
            r = await (await c.post("/v1/devices/offline",
                                    json={"device_id": "node1:gpu1", "reason": "hip"})).json()
            assert r["released"] == 3 and st.circuit.status("node1:gpu1") == "degraded"
            d = await (await c.get("/v1/dashboard")).json()
            trips = {x["id"]: x["circuit_trips"] for x in d["devices"]}
            assert trips.get("node1:gpu1") == 1
            # a worker re-registering for the engine device (after a
            # supervisor restart) brings it back online
            r = await c.post("/v1/workers/register", json={"worker": {
                "id": "worker-x", "tags": {"device_id": "node1:gpu1", "engine": True}}})
            assert r.status == 200
            assert st.store.get_device("node1:gpu1")["status"] == "online"
    run(go())


def test_llm_request_routing_and_deadline():
    async def go():
        st, c = client()
        async with c:
            r = await c.post("/v1/llm/request", json={"prompt": "hello", "model": "llama-3-8b"})
            j = await r.json()
            assert r.status == 202 and j["provider"] == "local" and j["kind"] == "engine.generate"
            r = await c.post("/v1/llm/request", json={"prompt": "hi", "provider": "ollama"})
            assert (await r.json())["kind"] == "ollama.generate"
            r = await c.post("/v1/llm/request", json={"task": "embed", "prompt": "hi"})
            assert (await r.json())["kind"] == "engine.embed"
            r = await c.post("/v1/llm/request", json={"quality": "bogus", "prompt": "x"})
            assert r.status == 400 and (await r.json())["error"] == "routing_failed"
            # smart routing needs a served local model of the right tier
            st.store.upsert_device("node1:gpu0", tags={"engine": True}, status="online")
            st.store.upsert_model("llama-3-8b", provider="local", kind="chat", tier="large",
                                  params_b=8.0, context_k=8)
            st.store.upsert_device_model("node1:gpu0", "llama-3-8b")
            r = await c.post("/v1/llm/request", json={"quality": "premium", "prompt": "hello"})
            j = await r.json()
            assert r.status == 202 and j["provider"] == "local"
            job = st.store.get_job(j["job_id"])
            assert job["payload"]["model"] == "llama-3-8b"
            assert job["payload"]["device_id"] == "node1:gpu0"
            assert job["payload"]["_tier"] == "large"
            assert 85 < job["deadline_at"] - time.time() <= 90
    run(go())


def test_costs_feedback_stats_benchmarks():
    async def go():
        st, c = client()
        async with c:
            st.store.set_pricing("m1", 1.0, 2.0)
            st.store.insert_cost(None, "m1", "openrouter", 1000, 1000,
                                 st.store.calculate_job_cost("m1", 1000, 1000))
            s = await (await c.get("/v1/costs/summary?period=week")).json()
            assert abs(s["total_cost"] - 0.003) < 1e-9 and s["total_jobs"] == 1
            assert s["by_provider"][0]["provider"] == "openrouter"
            assert (await c.get("/v1/costs/summary?period=year")).status == 400
            b = await (await c.get("/v1/costs/balance")).json()
            assert b["openrouter_balance_usd"] is None and b["top_models"][0]["model"] == "m1"
            r = await c.post("/v1/feedback", json={"model": "m1", "rating": "good"})
            assert (await r.json()) == {"status": "ok", "model": "m1", "rating": "good"}
            assert (await c.post("/v1/feedback", json={"model": "m1", "rating": "meh"})).status == 400
            ms = await (await c.get("/v1/models/stats")).json()
            assert ms["count"] == 1 and ms["models"][0]["feedback_score"] == 100.0
            r = await c.post("/v1/benchmarks/run", json={"model": "llama-3-8b", "runs": 2})
            j = await r.json()
            assert r.status == 202 and len(j["job_ids"]) == 2 and j["kind"] == "benchmark.engine.generate"
            st.store.insert_benchmark("d", "llama-3-8b", "generate", 10, 20, 100, 200.0)
            items = (await (await c.get("/v1/benchmarks?limit=5")).json())["items"]
            assert items[0]["tps"] == 200.0
            r = await c.post("/v1/knowledge/ingest", json={"text": "short", "target": "lightrag"})
            assert (await r.json())["error"] == "text_too_short"
    run(go())


def test_gpu_telemetry_from_drm_sysfs(tmp_path):
    """gpu_hbm_used_bytes / gpu_util come from the amdgpu DRM sysfs files."""
    from llm_mcp_amd.devices import rocm_enum
    for i, (busy, used, vendor) in enumerate([(37, 123456789, "0x1002"), (5, 7, "0x8086")]):
        pci = tmp_path / f"pci0000:00/0000:0{i + 3}:00.0"
        pci.mkdir(parents=True)
        (pci / "vendor").write_text(vendor + "\n")
        (pci / "gpu_busy_percent").write_text(f"{busy}\n")
        (pci / "mem_info_vram_used").write_text(f"{used}\n")
        card = tmp_path / "drm" / f"card{i}"
        card.mkdir(parents=True)
        (card / "device").symlink_to(pci)
    t = rocm_enum.gpu_telemetry(str(tmp_path / "drm"))
    assert t == {0: {"busy_pct": 37, "hbm_used_bytes": 123456789}}


def test_maintenance_exports_live_allreduce_samples():
    """rccl_allreduce_seconds takes the TP engine's start-up probe once and
    every new in-service sample (engine._comm_probe, seq-numbered) once."""
    from llm_mcp_amd.api.registry import LocalModel
    st = CoreState(store=MemoryStore())
    lm = LocalModel("llama-3-70b", "chat", "tp8-0", None, None, None,
                    tags={"tp_comm": {"rccl": {1 << 20: 40.0}},
                          "live": {"tp_comm_live": {"seq": 1, "us": {"rccl": 35.0, "peer": 12.0}}}})
    st.registry.add(lm)

    def count(path):
        for mf in st.metrics.allreduce.collect():
            for s in mf.samples:
                if s.name.endswith("_count") and s.labels.get("group") == path:
                    return s.value
        return 0.0
    st._maintenance()
    assert count("rccl") == 2 and count("peer") == 1
    st._maintenance()                                  # same samples: not re-observed
    assert count("rccl") == 2
    lm.tags["live"] = {"tp_comm_live": {"seq": 2, "us": {"rccl": 33.0}}}
    st._maintenance()
    assert count("rccl") == 3


def test_dashboard_counts_are_native_and_match_rows():
    """The dashboard's benchmark counts and per-device 7-day stats come from
    the native queue (no per-row conversion on every poll) and agree with a
    count over the rows."""
    from llm_mcp_amd.store.memory import MemoryStore
    st = MemoryStore()
    ids = [st.submit_job("benchmark.ollama.generate", {"model": "m"}) for _ in range(3)]
    ids += [st.submit_job("engine.generate", {"model": "m"}) for _ in range(2)]
    done = 0
    for _ in range(5):
        j = st.claim_job("w1", [], 30, worker_device="dev-a", check_online=False)
        if j is None:
            break
        if done < 3:
            st.complete_job(j["id"], "w1", {"ok": True}, {"ms": 100 + 10 * done},
                            j["attempt_id"])
        else:
            st.fail_job(j["id"], "w1", "boom", {"ms": 5}, j["attempt_id"])
        done += 1
    kc = st.kind_counts("benchmark.")
    rows = {}
    for s_ in ("queued", "running", "done", "error"):
        for r in st.list_jobs(s_, 0):
            if r["kind"].startswith("benchmark."):
                rows[s_] = rows.get(s_, 0) + 1
    assert {k: v for k, v in kc.items() if v} == rows
    stats = st.device_stats_7d("dev-a")
    # the two failed attempts were requeued (attempts < max_attempts): only
    # finished jobs count
    assert done == 5 and stats["total_jobs_7d"] == 3 and stats["done_jobs_7d"] == 3
    assert stats["avg_latency_ms"] == 110      # mean of 100, 110, 120


def test_job_change_hub_wakes_many_waiters_without_threads():
    """Hundreds of job streams / claim long-polls wait on one hub thread:
    one store change wakes all of them, and none holds an executor thread
    while it waits (routes.job_stream, routes._claim, rpc StreamJob)."""
    import threading
    from llm_mcp_amd.api.core import JobChangeHub

    async def go():
        st = CoreState(store=MemoryStore())
        hub = st.job_hub()
        assert st.job_hub() is hub
        v0 = hub.ver
        threads0 = threading.active_count()
        waiters = [asyncio.ensure_future(hub.wait(v0, 10.0)) for _ in range(300)]
        await asyncio.sleep(0.05)
        assert not any(w.done() for w in waiters)
        assert threading.active_count() == threads0      # no thread per waiter
        t = time.monotonic()
        await asyncio.to_thread(st.store.submit_job, "llm_generate", {"prompt": "x"})
        got = await asyncio.gather(*waiters)
        assert time.monotonic() - t < 2.0
        assert all(g != v0 for g in got) and len(set(got)) >= 1
        # a stale version returns at once; an unchanged one times out
        assert await hub.wait(v0, 5.0) == hub.ver
        t = time.monotonic()
        assert await hub.wait(hub.ver, 0.2) == hub.ver
        assert 0.15 < time.monotonic() - t < 1.5
        await st.stop_background()
        assert st._hub is None and not hub._thread.is_alive()
        assert isinstance(hub, JobChangeHub)
    run(go())


def test_active_jobs_on_is_indexed_and_tracks_transitions():
    """The router's per-device load (queued + running rows placed on a
    device) comes from an index kept by the native queue, not a row scan."""
    s = MemoryStore()
    s.upsert_device("gpu0", status="online")
    ids = [s.submit_job("llm_generate", {"device_id": "gpu0"}) for _ in range(3)]
    s.submit_job("llm_generate", {"device_id": "gpu1"})
    s.submit_job("llm_generate", {})
    assert s.active_jobs_on("gpu0") == 3 and s.active_jobs_on("gpu1") == 1
    j = s.claim_job("w", ["llm_generate"], 30, worker_device="gpu0", device_max_concurrency=0)
    assert j is not None and s.active_jobs_on("gpu0") == 3     # queued -> running
    assert s.complete_job(j["id"], "w", {}, {}, token=j.get("lease_token", ""))
    assert s.active_jobs_on("gpu0") == 2
    brute = sum(1 for st_ in ("queued", "running") for r in s.list_jobs(st_, 0)
                if r.get("device_id") == "gpu0")
    assert brute == s.active_jobs_on("gpu0") and ids
