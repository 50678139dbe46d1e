"""/v1/chat/completions (sync + SSE) end to end on the CPU engine."""
import asyncio
import json

import pytest
from aiohttp.test_utils import TestClient, TestServer

from llm_mcp_amd.api.app import ServingState, make_app
from llm_mcp_amd.api.registry import LocalModel, ModelRegistry
from llm_mcp_amd.engine.async_engine import AsyncEngine
from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine
from llm_mcp_amd.models.tokenizer import for_model
from llm_mcp_amd.utils.metrics import Metrics


@pytest.fixture(scope="module")
def engine():
    e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=8, max_batched_tokens=256,
                               max_model_len=512, use_graphs=False), device="cpu")
    yield e
    e.stop()


def _state(engine):
    aeng = AsyncEngine(engine)
    reg = ModelRegistry()
    reg.add(LocalModel("tiny-llama", "chat", "cpu0", aeng, for_model(engine.cfg), engine.cfg,
                       max_model_len=512, capacity=8))
    return ServingState(reg, Metrics()), aeng


def _run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def test_chat_sync_and_stream(engine):
    async def go():
        st, aeng = _state(engine)
        async with TestClient(TestServer(make_app(st))) as c:
            aeng.start(asyncio.get_running_loop())
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": [{"role": "user", "content": "hi there"}],
                "max_tokens": 5, "temperature": 0, "ignore_eos": True})
            assert r.status == 200
            j = await r.json()
            assert j["object"] == "chat.completion"
            assert j["usage"]["completion_tokens"] == 5
            assert j["choices"][0]["finish_reason"] == "length"
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": [{"role": "user", "content": "hi there"}],
                "max_tokens": 5, "temperature": 0, "ignore_eos": True, "stream": True,
                "stream_options": {"include_usage": True}},
                headers={"X-Request-ID": "chat-trace-1"})
            assert r.status == 200
            assert r.headers["Content-Type"].startswith("text/event-stream")
            assert r.headers["X-Request-ID"] == "chat-trace-1"
            body = (await r.read()).decode()
            frames = [f for f in body.split("\n\n") if f]
            assert frames[-1] == "data: [DONE]"
            chunks = [json.loads(f[6:]) for f in frames[:-1]]
            assert all(ch["object"] == "chat.completion.chunk" for ch in chunks)
            fin = [ch for ch in chunks if ch["choices"] and ch["choices"][0].get("finish_reason")]
            assert fin and fin[-1]["choices"][0]["delta"] == {}
            assert chunks[-1]["usage"]["completion_tokens"] == 5
            # same greedy text both ways
            text = "".join(ch["choices"][0]["delta"].get("content", "") for ch in chunks
                           if ch["choices"])
            assert text == j["choices"][0]["message"]["content"]
            # the stream's span is recorded under the client's request id
            tr = await (await c.get("/v1/debug/trace/chat-trace-1")).json()
            sp = tr["spans"][-1]
            assert sp["span"] == "chat" and sp["status"] == "ok"
            assert sp["completion_tokens"] == 5 and 0 <= sp["ttft_ms"] <= sp["total_ms"]
            # errors keep the reference contract
            r = await c.post("/v1/chat/completions", json={"model": "tiny-llama"})
            assert r.status == 400 and (await r.json())["error"] == "messages_required"
            r = await c.get("/v1/chat/completions")
            assert r.status == 405
            r = await c.post("/v1/chat/completions", json={
                "model": "nope", "messages": [{"role": "user", "content": "x"}]})
            assert r.status == 503 and (await r.json())["error"] == "no_device"
            r = await c.post("/v1/chat/completions", json={
                "model": "openai/gpt-4o", "messages": [{"role": "user", "content": "x"}]})
            assert r.status == 503 and (await r.json())["error"] == "cloud_disabled"
            m = await (await c.get("/metrics")).text()
            assert "llmcore_chat_requests_total" in m and "llm_ttft_seconds" in m
            aeng.stop()
    _run(go())


def test_stop_strings(engine):
    async def go():
        st, aeng = _state(engine)
        async with TestClient(TestServer(make_app(st))) as c:
            aeng.start(asyncio.get_running_loop())
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": [{"role": "user", "content": "abc"}],
                "max_tokens": 40, "temperature": 0, "ignore_eos": True})
            full = (await r.json())["choices"][0]["message"]["content"]
            assert len(full) > 4
            stop = full[2:4]
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": [{"role": "user", "content": "abc"}],
                "max_tokens": 40, "temperature": 0, "ignore_eos": True, "stop": [stop]})
            j = await r.json()
            assert j["choices"][0]["message"]["content"] == full[:full.index(stop)]
            assert j["choices"][0]["finish_reason"] == "stop"
            aeng.stop()
    _run(go())


def test_n_choices_sync_and_stream(engine):
    """OpenAI ``n``: n engine requests (seeds seed+i), choices by index; greedy
    choices agree, sampled ones differ; streamed chunks carry their index and
    every index gets its own finish chunk."""
    async def go():
        st, aeng = _state(engine)
        async with TestClient(TestServer(make_app(st))) as c:
            aeng.start(asyncio.get_running_loop())
            msg = [{"role": "user", "content": "tell me"}]
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": msg, "n": 3, "max_tokens": 6,
                "temperature": 0, "ignore_eos": True})
            j = await r.json()
            assert r.status == 200 and [ch["index"] for ch in j["choices"]] == [0, 1, 2]
            texts = {ch["message"]["content"] for ch in j["choices"]}
            assert len(texts) == 1 and j["usage"]["completion_tokens"] == 18
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": msg, "n": 4, "max_tokens": 12,
                "temperature": 1.5, "seed": 7, "ignore_eos": True})
            j = await r.json()
            assert len({ch["message"]["content"] for ch in j["choices"]}) > 1
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": msg, "n": 2, "max_tokens": 5,
                "temperature": 0.9, "ignore_eos": True, "stream": True,
                "stream_options": {"include_usage": True}})
            frames = [f for f in (await r.read()).decode().split("\n\n") if f]
            assert frames[-1] == "data: [DONE]"
            chunks = [json.loads(f[6:]) for f in frames[:-1]]
            fins = [ch["choices"][0]["index"] for ch in chunks
                    if ch["choices"] and ch["choices"][0].get("finish_reason")]
            assert sorted(fins) == [0, 1]
            assert chunks[-1]["usage"]["completion_tokens"] == 10
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": msg, "n": 0})
            assert r.status == 400 and (await r.json())["error"] == "invalid_n"
            aeng.stop()
    _run(go())


class _DeadEngine:
    """A replica whose worker died: every request fails before any token."""

    def __init__(self):
        self.calls = 0

    async def generate(self, prompt_ids, params, priority=0, stats=None):
        from llm_mcp_amd.engine.async_engine import StreamItem
        self.calls += 1
        yield StreamItem(-1, 0.0, "error:engine_disconnected")


def test_failover_before_first_token(engine):
    """Sync and streamed requests that land on a replica failing before its
    first token are resubmitted to a healthy replica (the breaker is fed);
    the client sees a normal completion."""
    from llm_mcp_amd.policy.circuit import CircuitBreaker

    async def go():
        st, aeng = _state(engine)
        dead = _DeadEngine()
        st.registry.add(LocalModel("tiny-llama", "chat", "dead0", dead, for_model(engine.cfg),
                                   engine.cfg, max_model_len=512, capacity=8))
        st.circuit = CircuitBreaker()
        async with TestClient(TestServer(make_app(st))) as c:
            aeng.start(asyncio.get_running_loop())
            for stream in (False, True, False):
                # make the dead replica the least loaded one so it is picked first
                for m in st.registry.replicas("tiny-llama"):
                    m.inflight = 0 if m.device_id == "dead0" else 1
                r = await c.post("/v1/chat/completions", json={
                    "model": "tiny-llama", "messages": [{"role": "user", "content": "hi"}],
                    "max_tokens": 5, "temperature": 0, "ignore_eos": True, "stream": stream})
                assert r.status == 200
                body = await r.text()
                if stream:
                    assert '"finish_reason":"length"' in body.replace(" ", "") and \
                        body.rstrip().endswith("[DONE]")
                else:
                    assert json.loads(body)["usage"]["completion_tokens"] == 5
            assert dead.calls >= 2
            assert st.circuit.status("dead0") in ("degraded", "probe", "ok")
    _run(go())


class _DiesMidway:
    """A replica that streams two tokens, then loses its worker."""

    async def generate(self, prompt_ids, params, priority=0, stats=None):
        from llm_mcp_amd.engine.async_engine import StreamItem
        yield StreamItem(7, 0.0, None)
        yield StreamItem(8, 0.0, None)
        yield StreamItem(-1, 0.0, "error:engine_disconnected")


def test_sync_request_restarts_after_midway_failure(engine):
    """A non-streaming request is buffered until the end, so a replica dying
    mid-generation costs a restart on another replica, not an error."""
    async def go():
        st, aeng = _state(engine)
        st.registry.add(LocalModel("tiny-llama", "chat", "flaky0", _DiesMidway(),
                                   for_model(engine.cfg), engine.cfg, max_model_len=512,
                                   capacity=8))
        async with TestClient(TestServer(make_app(st))) as c:
            aeng.start(asyncio.get_running_loop())
            for m in st.registry.replicas("tiny-llama"):
                m.inflight = 0 if m.device_id == "flaky0" else 1
            r = await c.post("/v1/chat/completions", json={
                "model": "tiny-llama", "messages": [{"role": "user", "content": "hi"}],
                "max_tokens": 6, "temperature": 0, "ignore_eos": True})
            body = await r.json()
            assert r.status == 200, body
            assert body["usage"]["completion_tokens"] == 6
    _run(go())
