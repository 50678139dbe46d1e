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
    # request id via call metadata lands in the payload
    j3 = c.submit("echo", {"a": 1}, request_id="grpc-trace-1")
    assert c.get(j3)["payload"] == {"a": 1, "_request_id": "grpc-trace-1"}


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


def test_server_reflection_lists_and_describes_core():
    import asyncio
    import threading
    import time

    import grpc
    from google.protobuf import descriptor_pb2

    from llm_mcp_amd.api.core import CoreState
    from llm_mcp_amd.rpc import proto as pb
    from llm_mcp_amd.rpc.server import start_grpc
    from llm_mcp_amd.store.memory import MemoryStore

    loop = asyncio.new_event_loop()
    box = {}

    def run():
        asyncio.set_event_loop(loop)
        box["srv"], box["port"] = loop.run_until_complete(
            start_grpc(CoreState(store=MemoryStore()), "127.0.0.1:0"))
        loop.run_forever()

    threading.Thread(target=run, daemon=True).start()
    while "port" not in box:
        time.sleep(0.01)
    R = pb.reflection
    ch = grpc.insecure_channel(f"127.0.0.1:{box['port']}")
    call = ch.stream_stream(f"/{pb.REFLECTION_SERVICE}/ServerReflectionInfo",
                            request_serializer=R["ServerReflectionRequest"].SerializeToString,
                            response_deserializer=R["ServerReflectionResponse"].FromString)
    reqs = [R["ServerReflectionRequest"](list_services="*"),
            R["ServerReflectionRequest"](file_containing_symbol="llmmcp.v1.Core"),
            R["ServerReflectionRequest"](file_containing_symbol="nope.Nothing")]
    out = list(call(iter(reqs)))
    names = [s.name for s in out[0].list_services_response.service]
    assert "llmmcp.v1.Core" in names
    fd = descriptor_pb2.FileDescriptorProto.FromString(
        out[1].file_descriptor_response.file_descriptor_proto[0])
    assert fd.package == "llmmcp.v1" and "ClaimJob" in [m.name for m in fd.service[0].method]
    assert out[2].error_response.error_code == grpc.StatusCode.NOT_FOUND.value[0]
    ch.close()
    loop.call_soon_threadsafe(loop.stop)
