"""API process <-> engine process link (Unix socket, msgpack) on the CPU engine."""
import asyncio
import json
import os
import tempfile

from aiohttp.test_utils import TestClient, TestServer

from llm_mcp_amd.api.app import ServingState, make_app
from llm_mcp_amd.api.registry import ModelRegistry
from llm_mcp_amd.api.serve import attach_engines, parse_engine_spec
from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine
from llm_mcp_amd.engine.ipc import EngineServer
from llm_mcp_amd.utils.metrics import Metrics


def test_chat_over_ipc():
    e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=8, max_batched_tokens=256,
                               max_model_len=512, use_graphs=False), device="cpu")
    path = os.path.join(tempfile.mkdtemp(), "eng.sock")
    srv = EngineServer(e, path, info={"kind": "chat", "max_model_len": 512, "capacity": 8})
    srv.start()

    async def go():
        st = ServingState(ModelRegistry(), Metrics())
        await attach_engines(st, [parse_engine_spec(f"tiny-llama=unix:{path},device=cpu0")])
        m = st.registry.select("tiny-llama", "chat")
        assert m is not None and m.max_model_len == 512 and m.device_id == "cpu0"
        async with TestClient(TestServer(make_app(st))) as c:
            outs = []
            for stream in (False, True):
                r = await c.post("/v1/chat/completions", json={
                    "model": "tiny-llama", "messages": [{"role": "user", "content": "hello"}],
                    "max_tokens": 6, "temperature": 0, "ignore_eos": True, "stream": stream})
                assert r.status == 200
                if stream:
                    frames = [f for f in (await r.read()).decode().split("\n\n") if f]
                    assert frames[-1] == "data: [DONE]"
                    outs.append("".join(json.loads(f[6:])["choices"][0]["delta"].get("content", "")
                                        for f in frames[:-1]))
                else:
                    outs.append((await r.json())["choices"][0]["message"]["content"])
            assert outs[0] == outs[1]
            # many concurrent streams over one connection
            rs = await asyncio.gather(*[c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": [{"role": "user", "content": f"q{i}"}],
                "max_tokens": 4, "temperature": 0.7, "ignore_eos": True}) for i in range(12)])
            for r in rs:
                assert (await r.json())["usage"]["completion_tokens"] == 4
            info = await m.engine.info()
            assert info["stats"]["finished"] >= 14

    try:
        asyncio.new_event_loop().run_until_complete(go())
    finally:
        srv.stop()


def test_embeddings_over_ipc_api_process_app():
    """The API-only process (api/serve.py) serves /v1/embeddings from an
    embedding engine living in another process's EngineServer."""
    from llm_mcp_amd.api.serve import make_serving_app
    from llm_mcp_amd.engine.embed_engine import EmbeddingEngine
    from llm_mcp_amd.models import config as mc
    emb = EmbeddingEngine(mc.resolve("tiny-nomic"), device="cpu")
    path = os.path.join(tempfile.mkdtemp(), "emb.sock")
    srv = EngineServer(None, path, info={"models": {"tiny-nomic": {
        "kind": "embed", "max_model_len": 512, "capacity": 64}}}, embed_engine=emb)
    srv.start()

    async def go():
        app, st = make_serving_app([parse_engine_spec(f"tiny-nomic=unix:{path},device=cpu0")])
        async with TestClient(TestServer(app)) as c:
            for _ in range(100):
                if (await c.get("/ready")).status == 200:
                    break
                await asyncio.sleep(0.05)
            r = await c.post("/v1/embeddings", json={"model": "tiny-nomic",
                                                     "input": ["a doc", "another doc"],
                                                     "dimensions": 64})
            body = await r.json()
            assert r.status == 200, body
            assert len(body["data"]) == 2 and len(body["data"][0]["embedding"]) == 64
            assert body["usage"]["prompt_tokens"] > 0

    try:
        asyncio.new_event_loop().run_until_complete(go())
    finally:
        srv.stop()


def test_embedding_response_rows_are_exact_float32():
    """/v1/embeddings bodies are spliced from natively formatted rows
    (shortest float32 round trip): parsing them back gives the float32
    values bit for bit; non-finite values become null."""
    import json

    import numpy as np

    from llm_mcp_amd.api.openai_embed import _response
    from llm_mcp_amd.native import runtime
    v = (np.random.default_rng(0).standard_normal((5, 96)) * 10.0 ** np.arange(-6, 6, 0.125)[:96]
         ).astype(np.float32)
    body = json.loads(_response(v.tolist(), "float", "m", 7).text)
    assert [d["index"] for d in body["data"]] == list(range(5))
    back = np.asarray([d["embedding"] for d in body["data"]], np.float32)
    assert np.array_equal(back, v)
    assert body["usage"] == {"prompt_tokens": 7, "total_tokens": 7}
    row = json.loads(runtime().f32_json_rows(np.asarray([[1.5, np.nan, -np.inf, 0.0]],
                                                        np.float32))[0])
    assert row == [1.5, None, None, 0.0]


def test_engine_info_survives_strict_msgpack_with_tp_probe_sizes():
    """A TP leader's start-up all-reduce probe is keyed by message size
    (ints): the engine socket's peer unpacks with msgpack's strict_map_key,
    so the info reply must carry those keys as strings (a GPU TP group's
    info request used to drop the connection)."""
    import types

    import msgpack

    from llm_mcp_amd.engine.ipc import EngineServer
    sched = types.SimpleNamespace(num_running=1, num_waiting=0, kv_usage=0.5, kv_free_blocks=7)
    eng = types.SimpleNamespace(sched=sched, stats={"steps": 3},
                                tp_comm={"rccl": {16384: 21.5, 1048576: 80.0}, "peer": {16384: 9.1}},
                                tp_comm_live={"seq": 2, "bytes": 1 << 20, "us": {"rccl": 75.0}})
    srv = EngineServer.__new__(EngineServer)
    srv.engine = eng
    info = srv.engine_info()
    back = msgpack.unpackb(msgpack.packb(info), raw=False)
    assert back["tp_comm"]["rccl"]["16384"] == 21.5 and back["tp_comm_live"]["us"]["rccl"] == 75.0
