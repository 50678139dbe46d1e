"""Fault injection: injected job crashes are retried through
the lease queue until they succeed or exhaust their attempts; a dropped claim
is recovered after its lease expires; an unhealthy engine stops extending
leases and reports its device offline; an injected GPU error fails the
in-flight requests without killing the engine."""
import asyncio
import time

from llm_mcp_amd.api.registry import ModelRegistry
from llm_mcp_amd.engine.engine import EngineConfig, GenRequest, LLMEngine, SamplingParams
from llm_mcp_amd.store.memory import MemoryStore
from llm_mcp_amd.utils.faults import Faults, set_faults
from llm_mcp_amd.worker.agent import WorkerAgent
from llm_mcp_amd.worker.jobs import JobRunner


class StoreClient:
    """CoreClient stand-in backed directly by a store (same call surface)."""

    def __init__(self, store):
        self.s = store

    def register(self, worker_id, name, platform, arch, host, tags):
        self.s.upsert_device(worker_id or "worker-x", name=name, tags=tags)
        return worker_id or "worker-x"

    def claim(self, worker_id, kinds, lease_s, device_id, wait_ms):
        j = self.s.claim_job(worker_id, kinds, lease_s, worker_device=device_id,
                             check_online=False)
        if j is None:
            time.sleep(0.01)
        return j

    def heartbeat(self, worker_id, jid, extend, token):
        return self.s.heartbeat(jid, worker_id, extend, token)

    def complete(self, worker_id, jid, result, metrics, token):
        return self.s.complete_job(jid, worker_id, result, metrics, token)

    def fail(self, worker_id, jid, err, metrics, token):
        return self.s.fail_job(jid, worker_id, err, metrics, token)


def test_injected_job_crashes_are_retried():
    st = MemoryStore()
    ids = [st.submit_job("echo", {"i": i}, max_attempts=6) for i in range(40)]
    set_faults(Faults("job_crash:0.3", seed=1))
    try:
        agent = WorkerAgent(StoreClient(st), JobRunner(ModelRegistry(), "d0"), "d0",
                            worker_id="worker-a", lease_s=30, capacity=4)

        async def go():
            task = asyncio.create_task(agent.run())
            for _ in range(400):
                c = st.job_counts()
                if c.get("queued", 0) + c.get("running", 0) == 0:
                    break
                await asyncio.sleep(0.02)
            agent.stop()
            await task
        asyncio.new_event_loop().run_until_complete(go())
    finally:
        set_faults(None)
    done = sum(st.get_job(i)["status"] == "done" for i in ids)
    assert agent.stats["failed"] > 0 and done >= 38
    crashed = [i for i in ids if len(st.job_attempts(i)) > 1]
    assert crashed and all(st.get_job(i)["attempts"] == len(st.job_attempts(i)) for i in crashed)


def test_dropped_claim_recovers_after_lease_expiry():
    t = [1000.0]
    st = MemoryStore(clock=lambda: t[0])
    jid = st.submit_job("echo", {"x": 1})
    j = st.claim_job("w-dead", [], 10)          # a worker that vanished with its lease
    assert j and st.claim_job("w2", [], 10) is None
    t[0] += 11
    j2 = st.claim_job("w2", [], 10)
    assert j2["id"] == jid and j2["attempts"] == 2
    assert st.complete_job(jid, "w2", {"ok": True}, {}, j2["attempt_id"])
    assert not st.complete_job(jid, "w-dead", {"ok": False}, {}, j["attempt_id"])


def test_unhealthy_engine_stops_heartbeats_and_reports_offline():
    st = MemoryStore()
    st.upsert_device("d0", name="gpu0", status="online")
    offline = []
    agent = WorkerAgent(StoreClient(st), JobRunner(ModelRegistry(), "d0"), "d0",
                        worker_id="worker-b", lease_s=1, capacity=1,
                        mark_offline=lambda dev, why: offline.append((dev, why)),
                        health=lambda: (False, "engine step running for 130s"))
    beats = []
    agent.client.heartbeat = lambda *a: beats.append(a) or True

    async def go():
        hb = asyncio.create_task(agent._heartbeat("job", "tok"))
        await asyncio.sleep(5.5)
        hb.cancel()
    asyncio.new_event_loop().run_until_complete(go())
    assert beats == [] and offline and offline[0][0] == "d0"


def test_injected_gpu_error_fails_requests_engine_survives():
    e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=4, max_batched_tokens=64,
                               max_model_len=256, use_graphs=False), device="cpu")
    evs = []
    e.event_sink = evs.extend
    set_faults(Faults("gpu_error:1.0"))
    e.start()
    try:
        e.submit(GenRequest([1, 2, 3], SamplingParams(max_tokens=3)))
        for _ in range(200):
            if any(ev.finish == "engine_error" or (ev.finish or "").startswith("error")
                   for ev in evs):
                break
            time.sleep(0.01)
        set_faults(None)
        assert any((ev.finish or "").endswith("error") for ev in evs)
        ok, why = e.healthy()
        assert not ok and "HIP error" in why
        # the engine thread is still serving
        evs.clear()
        e._last_error = None
        e.submit(GenRequest([4, 5], SamplingParams(max_tokens=2, ignore_eos=True)))
        for _ in range(500):
            if any(ev.finish for ev in evs):
                break
            time.sleep(0.01)
        assert [ev.finish for ev in evs if ev.finish] == ["length"]
    finally:
        set_faults(None)
        e.stop()


def test_fault_schedule_fires_at_fixed_calls():
    from llm_mcp_amd.utils.faults import Faults
    f = Faults("gpu_error@3/5,job_crash:0.0")
    fired = [f.hit("gpu_error") for _ in range(7)]
    assert fired == [False, False, True, False, True, False, False]
    assert f.fired["gpu_error"] == 2 and not f.hit("job_crash") and bool(f)
    g = Faults("gpu_error@3/5")
    assert [g.hit("gpu_error") for _ in range(7)] == fired     # same schedule every process
