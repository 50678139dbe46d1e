"""submit -> claim -> heartbeat -> complete with the GPU worker agent running
its in-process engines on CPU (BASELINE config 1: plumbing, no GPU)."""
import asyncio
import threading
import time

import pytest

from llm_mcp_amd.api.core import CoreState
from llm_mcp_amd.api.registry import LocalModel, ModelRegistry
from llm_mcp_amd.engine.async_engine import AsyncEngine
from llm_mcp_amd.engine.embed_engine import EmbeddingEngine
from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine
from llm_mcp_amd.models import config as mc
from llm_mcp_amd.models.tokenizer import for_model
from llm_mcp_amd.rpc.client import CoreClient
from llm_mcp_amd.rpc.server import start_grpc
from llm_mcp_amd.store.memory import MemoryStore
from llm_mcp_amd.worker.agent import WorkerAgent
from llm_mcp_amd.worker.jobs import JobRunner


@pytest.fixture(scope="module")
def core():
    st = CoreState(store=MemoryStore())
    loop = asyncio.new_event_loop()
    box = {}

    def run():
        asyncio.set_event_loop(loop)
        box["srv"], box["port"] = loop.run_until_complete(start_grpc(st, "127.0.0.1:0"))
        loop.run_forever()

    threading.Thread(target=run, daemon=True).start()
    while "port" not in box:
        time.sleep(0.01)
    yield st, f"127.0.0.1:{box['port']}"
    loop.call_soon_threadsafe(loop.stop)


def test_worker_executes_engine_jobs(core):
    st, addr = core
    client = CoreClient(addr)
    eng = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=8, max_batched_tokens=256,
                                 max_model_len=512, use_graphs=False), device="cpu")
    emb = EmbeddingEngine(mc.resolve("tiny-nomic"), device="cpu")

    async def go():
        aeng = AsyncEngine(eng)
        aeng.start(asyncio.get_running_loop())
        emb.start()
        reg = ModelRegistry()
        reg.add(LocalModel("tiny-llama", "chat", "n:gpu0", aeng, for_model(eng.cfg), eng.cfg,
                           512, 8))
        reg.add(LocalModel("tiny-nomic", "embed", "n:gpu0", emb, for_model(emb.cfg), emb.cfg,
                           512, 64))
        runner = JobRunner(reg, "n:gpu0",
                           report_benchmark=lambda **kw: client.report_benchmark(**kw))
        st.store.set_pricing("tiny-llama", 1.0, 2.0)
        ids = {
            "gen": client.submit("engine.generate", {"model": "tiny-llama", "prompt": "hello",
                                                      "options": {"max_tokens": 5,
                                                                  "temperature": 0,
                                                                  "ignore_eos": True},
                                                      "_price_in_1m": 1.0,
                                                      "_price_out_1m": 2.0}),
            "alias": client.submit("ollama.generate", {"model": "tiny-llama",
                                                        "messages": [{"role": "user",
                                                                      "content": "hi"}],
                                                        "options": {"max_tokens": 3}}),
            "emb": client.submit("engine.embed", {"model": "tiny-nomic", "prompt": "doc"}),
            "bench": client.submit("benchmark.engine.generate",
                                   {"model": "tiny-llama", "max_tokens": 8, "prompt_tokens": 16,
                                    "concurrency": 2}),
            "echo": client.submit("echo", {"a": 1}),
        }
        agent = WorkerAgent(client, runner, "n:gpu0", lease_s=30, capacity=8)
        await agent.run(max_jobs=len(ids))
        aeng.stop()
        emb.stop()
        return ids, agent

    ids, agent = asyncio.new_event_loop().run_until_complete(go())
    jobs = {k: client.get(v) for k, v in ids.items()}
    assert all(j["status"] == "done" for j in jobs.values()), jobs
    g = jobs["gen"]["result"]
    assert g["ok"] and g["provider"] == "local" and g["tokens_out"] == 5 and g["device_id"] == "n:gpu0"
    assert g["cost"].endswith("$") and float(g["cost"][:-1]) > 0
    assert jobs["alias"]["result"]["tokens_out"] <= 3
    assert len(jobs["emb"]["result"]["data"]["embedding"]) == 256
    b = jobs["bench"]["result"]
    assert b["tokens_out"] == 16 and b["tps"] > 0
    assert st.store.list_benchmarks(1)[0]["model_id"] == "tiny-llama"
    assert jobs["echo"]["result"] == {"ok": True, "echo": {"a": 1}}
    # RecordCost on the gRPC completion path (reference gap fixed)
    assert st.store.cost_summary(0)["total_jobs"] >= 1
    assert agent.stats["done"] == 5


def test_progress_over_grpc_and_agent(core):
    """CoreClient.progress (a Heartbeat with progress_json) lands on the job;
    the agent forwards a running job's progress dict while it changes."""
    st, addr = core
    client = CoreClient(addr)
    jid = client.submit("prog.test", {})
    j = client.claim("w-prog", ["prog.test"], 30, "", 0)
    assert j and j["id"] == jid
    assert client.progress("w-prog", jid, {"tokens_out": 7}, 30, j["attempt_id"])
    assert st.store.get_job(jid)["progress"] == {"tokens_out": 7}
    assert not client.progress("w-prog", jid, {"tokens_out": 8}, 30, "stale-token")
    assert client.complete("w-prog", jid, {"ok": True}, {}, j["attempt_id"])

    class Ticking:
        async def handle(self, kind, payload, progress=None):
            for n in range(1, 4):
                progress["tokens_out"] = n
                await asyncio.sleep(0.15)
            return {"ok": True}, {"ms": 1}

    async def go():
        jid2 = client.submit("prog.agent", {})
        agent = WorkerAgent(client, Ticking(), "n:gpu3", kinds=["prog.agent"], lease_s=30,
                            capacity=2, progress_s=0.05)
        await agent.run(max_jobs=1)
        return jid2, agent
    jid2, agent = asyncio.new_event_loop().run_until_complete(go())
    assert agent.stats["progress_sent"] >= 2
    assert client.get(jid2)["status"] == "done"


def test_admission_gate_leaves_jobs_for_other_workers(core):
    """A worker whose engine reports no headroom keeps at most the jobs it
    already holds; the rest stay queued and are claimed by another worker
    (admission by engine capacity, not a fixed per-device concurrency)."""
    st, addr = core
    client = CoreClient(addr)

    class Slow:
        """Stands in for a JobRunner: holds every job until released."""
        def __init__(self):
            self.release = asyncio.Event()
            self.seen = 0

        async def handle(self, kind, payload, progress=None):
            self.seen += 1
            await self.release.wait()
            return {"ok": True}, {"ms": 1}

    for dev in ("n:gpu1", "n:gpu2"):   # GPU devices admit their batching capacity
        st.store.upsert_device(dev, name=dev, tags={"capacity": 8})

    async def go():
        ids = [client.submit("gate.test", {"i": i}) for i in range(6)]
        busy, free = Slow(), Slow()
        gated = {"n": 0}

        def admit():          # the "busy" GPU: full after its first job
            gated["n"] += 1
            return False, "kv cache 97% full"
        a = WorkerAgent(client, busy, "n:gpu1", kinds=["gate.test"], lease_s=30, capacity=8,
                        admit=admit)
        b = WorkerAgent(client, free, "n:gpu2", kinds=["gate.test"], lease_s=30, capacity=8)
        ta = asyncio.ensure_future(a.run())
        await asyncio.sleep(0.5)          # a claims one job, then the gate closes
        assert busy.seen == 1 and gated["n"] > 0
        tb = asyncio.ensure_future(b.run(max_jobs=5))
        for _ in range(100):
            if free.seen == 5:
                break
            await asyncio.sleep(0.05)
        assert free.seen == 5 and busy.seen == 1
        busy.release.set()
        free.release.set()
        await tb
        a.stop()
        await asyncio.wait_for(ta, 10)
        return ids
    ids = asyncio.new_event_loop().run_until_complete(go())
    assert all(client.get(i)["status"] == "done" for i in ids)
