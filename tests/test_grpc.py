"""llmmcp.v1.Core over gRPC (runtime-built descriptors) against the memory store."""
import asyncio
import threading
import time

import pytest

from llm_mcp_amd.api.core import CoreState
from llm_mcp_amd.rpc.client import CoreClient
from llm_mcp_amd.rpc.server import start_grpc
from llm_mcp_amd.store.memory import MemoryStore


@pytest.fixture
def core():
    st = CoreState(store=MemoryStore())
    loop = asyncio.new_event_loop()
    box = {}

    def run():
        asyncio.set_event_loop(loop)
        srv, port = loop.run_until_complete(start_grpc(st, "127.0.0.1:0"))
        box["srv"], box["port"] = srv, port
        loop.run_forever()

    t = threading.Thread(target=run, daemon=True)
    t.start()
    while "port" not in box:
        time.sleep(0.01)
    c = CoreClient(f"127.0.0.1:{box['port']}")
    yield st, c
    c.close()
    asyncio.run_coroutine_threadsafe(box["srv"].stop(None), loop).result(5)
    loop.call_soon_threadsafe(loop.stop)


def test_grpc_worker_protocol(core):
    st, c = core
    wid = c.register(name="gpu-worker", platform="rocm", arch="gfx950", tags={"engine": True})
    assert wid.startswith("worker-")
    jid = c.submit("echo", {"hello": 1}, priority=5, source="test")
    assert c.get(jid)["status"] == "queued"
    j = c.claim(wid, ["echo"], 30)
    assert j["id"] == jid and j["attempt_id"] and j["payload"] == {"hello": 1}
    assert c.claim(wid, ["echo"], 30) is None
    assert c.heartbeat(wid, jid, 30, j["attempt_id"])
    assert not c.complete(wid, jid, {"x": 1}, attempt_id="stale")
    assert c.complete(wid, jid, {"ok": True}, {"tokens_in": 1, "tokens_out": 2,
                                               "provider": "local", "model": "m"},
                      attempt_id=j["attempt_id"])
    got = c.get(jid)
    assert got["status"] == "done" and got["result"] == {"ok": True}
    events = list(c.stream(jid))
    assert events[-1]["message"] == "done"
    j2 = c.submit("echo", {}, max_attempts=1)
    a = c.claim(wid, [], 30)
    assert c.fail(wid, j2, "boom", attempt_id=a["attempt_id"]) == "error"
    assert c.report_benchmark("dev0", "llama-3-8b", "generate", 10, 100, 500, 200.0)
    assert st.store.list_benchmarks(1)[0]["tps"] == 200.0
    assert c.report_metrics({"id": wid, "name": "w"}, {"gpu_util": 90})


def test_grpc_claim_long_poll_wakes_on_submit(core):
    st, c = core
    out = {}

    def claimer():
        t0 = time.time()
        out["job"] = c.claim("w", [], 30, wait_ms=5000)
        out["dt"] = time.time() - t0

    th = threading.Thread(target=claimer)
    th.start()
    time.sleep(0.3)
    jid = c.submit("k", {})
    th.join(10)
    assert out["job"]["id"] == jid and out["dt"] < 3.0
