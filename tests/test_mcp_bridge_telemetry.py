"""MCP JSON-RPC tool server, HTTP bridge and telemetry alert loop."""
import asyncio
import io
import json

import pytest
from aiohttp.test_utils import TestClient, TestServer

from llm_mcp_amd.api.core import CoreState, create_core_app
from llm_mcp_amd.mcp.bridge import make_bridge, submit_request
from llm_mcp_amd.mcp.server import TOOLS, MCPServer, build_call
from llm_mcp_amd.store.memory import MemoryStore
from llm_mcp_amd.telemetry.alerts import AlertLoop, format_alert, snapshot_from_store


def run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def test_reference_tool_names_present():
    ref = ["llm_dashboard", "llm_submit", "llm_job_status", "llm_request", "llm_costs",
           "llm_benchmarks", "llm_balance", "llm_model_stats", "llm_feedback", "llm_learn",
           "llm_remember", "llm_sync_models"]
    assert all(t in TOOLS for t in ref)


def test_mcp_jsonrpc_protocol():
    srv = MCPServer("http://127.0.0.1:1")

    async def go():
        r = await srv.handle({"jsonrpc": "2.0", "id": 1, "method": "initialize", "params": {}})
        assert r["result"]["capabilities"]["tools"] is not None
        assert await srv.handle({"jsonrpc": "2.0", "method": "notifications/initialized"}) is None
        r = await srv.handle({"jsonrpc": "2.0", "id": 2, "method": "tools/list"})
        names = {t["name"] for t in r["result"]["tools"]}
        assert "llm_chat" in names and "llm_submit" in names
        r = await srv.handle({"jsonrpc": "2.0", "id": 3, "method": "nope"})
        assert r["error"]["code"] == -32601
        r = await srv.handle({"jsonrpc": "2.0", "id": 4, "method": "tools/call",
                              "params": {"name": "llm_dashboard", "arguments": {}}})
        assert r["result"]["isError"] is True  # backend unreachable -> tool error, not crash
        if srv._session:
            await srv._session.close()
    run(go())

    # stdio transport
    inp = io.StringIO(json.dumps({"jsonrpc": "2.0", "id": 9, "method": "ping"}) + "\n")
    out = io.StringIO()
    run(MCPServer("http://x").serve_stdio(inp, out))
    assert json.loads(out.getvalue())["result"] == {}


def test_llm_submit_is_a_generation_job_not_echo():
    method, path, body, _ = build_call("llm_submit", {"model": "llama-3-8b", "prompt": "hi"})
    kind, payload, _ = submit_request(body)
    assert kind == "engine.generate" and payload["prompt"] == "hi"
    assert submit_request({"kind": "echo", "payload": {"a": 1}})[0] == "echo"


class FakeGrpc:
    def __init__(self, store):
        self.store = store

    def submit(self, kind, payload, prio=0, source=""):
        return self.store.submit_job(kind, payload, prio, source)

    def get(self, jid):
        j = self.store.get_job(jid)
        if j is None:
            raise KeyError(jid)
        return {"id": j["id"], "status": j["status"], "kind": j["kind"]}

    def stream(self, jid):
        j = self.store.get_job(jid)
        yield {"type": "status", "data": {"status": j["status"]}}


def test_bridge_routes_and_proxies():
    async def go():
        st = CoreState(store=MemoryStore())
        core = TestServer(create_core_app(st, background=False))
        await core.start_server()
        bridge = TestClient(TestServer(make_bridge(str(core.make_url("")), FakeGrpc(st.store))))
        async with bridge:
            assert (await (await bridge.get("/health")).json())["status"] == "ok"
            r = await bridge.post("/submit", json={"model": "llama-3-8b", "prompt": "hello"})
            j = await r.json()
            assert r.status == 202 and j["kind"] == "engine.generate"
            assert (await (await bridge.get(f"/jobs/{j['job_id']}")).json())["status"] == "queued"
            body = (await (await bridge.get(f"/jobs/{j['job_id']}/stream")).read()).decode()
            assert body.startswith("event: status\ndata: ")
            d = await bridge.get("/dashboard")
            assert d.status == 200 and "hosts" in await d.json()
            disc = await bridge.get("/discovery")
            assert disc.status == 200 and "last_run" in await disc.json()
            c = await bridge.get("/costs/summary?period=week")
            assert (await c.json())["period"] == "week"
        await core.close()
    run(go())


def test_telemetry_alerts_baseline_transitions_and_dedupe():
    st = MemoryStore()
    st.upsert_device("n:gpu0", name="gpu0", tags={"engine": True}, status="online")
    st.upsert_device("n:gpu1", name="gpu1", tags={"engine": True, "temp_c": 101.0},
                     status="online")
    snaps = []

    async def fetch():
        s = snapshot_from_store(st, fail_threshold=1)
        snaps.append(s)
        return s

    loop = AlertLoop(fetch, sinks=[])

    async def go():
        assert await loop.tick() is None  # baseline
        st.set_device_status("n:gpu0", "offline")
        jid = st.submit_job("engine.generate", {}, max_attempts=1)
        j = st.claim_job("w", [], 30)
        st.fail_job(jid, "w", "HIP error: illegal address", {}, j["attempt_id"])
        t = await loop.tick()
        assert "OFFLINE: gpu0" in t and "GPU hot: gpu1" in t and "Job failed" in t
        st.set_device_status("n:gpu0", "online")
        t2 = await loop.tick()
        assert "ONLINE: gpu0" in t2 and "Job failed" not in t2  # failed job deduped
    run(go())
    assert format_alert({"queued": 3, "running": 0, "devices": [], "failed_jobs": []},
                        set(), []).endswith("Queue stuck: 3 queued, 0 running")


def test_telegram_sinks_edit_in_place_and_gateway_fallback(monkeypatch):
    """Bot API sink: sendMessage once, then editMessageText of that message
    ("not modified" counts as sent, a vanished message is re-sent); gateway
    sink: POST then PATCH, falling back to the Bot API when it fails."""
    from aiohttp import web
    from aiohttp.test_utils import TestServer
    from llm_mcp_amd.telemetry import alerts as al

    calls = []
    state = {"gw_up": True, "next_edit": "ok"}

    async def bot(request):
        body = await request.json()
        method = request.match_info["method"]
        calls.append(("bot", method, body.get("message_id"), body["text"]))
        if method == "sendMessage":
            return web.json_response({"ok": True, "result": {"message_id": 100 + len(calls)}})
        mode, state["next_edit"] = state["next_edit"], "ok"
        if mode == "same":
            return web.json_response({"ok": False, "description":
                                      "Bad Request: message is not modified"}, status=400)
        if mode == "gone":
            return web.json_response({"ok": False, "description":
                                      "Bad Request: message to edit not found"}, status=400)
        return web.json_response({"ok": True, "result": {}})

    async def gw_post(request):
        body = await request.json()
        calls.append(("gw", "post", None, body["text"]))
        if not state["gw_up"]:
            return web.json_response({"error": "down"}, status=503)
        return web.json_response({"id": 7})

    async def gw_patch(request):
        calls.append(("gw", "patch", request.match_info["mid"], (await request.json())["text"]))
        if not state["gw_up"]:
            return web.json_response({"error": "down"}, status=503)
        return web.json_response({"ok": True})

    app = web.Application()
    app.router.add_post("/botTOK/{method}", bot)
    app.router.add_post("/api/messages", gw_post)
    app.router.add_patch("/api/messages/{mid}", gw_patch)

    async def go():
        srv = TestServer(app)
        await srv.start_server()
        base = str(srv.make_url("")).rstrip("/")
        try:
            direct = al.TelegramSink("TOK", "42", base=base)
            assert await direct.send_or_edit("a <b>")
            first = direct.last_id
            assert await direct.send_or_edit("b")
            state["next_edit"] = "same"
            assert await direct.send_or_edit("b")
            state["next_edit"] = "gone"
            assert await direct.send_or_edit("c")
            assert direct.last_id != first
            kinds = [(c[1], c[2]) for c in calls if c[0] == "bot"]
            assert kinds[0] == ("sendMessage", None) and kinds[1] == ("editMessageText", first)
            assert kinds[-2][0] == "editMessageText" and kinds[-1][0] == "sendMessage"
            assert calls[0][3] == "<pre>a &lt;b&gt;</pre>"

            calls.clear()
            g = al.GatewaySink(al.McpTelegramSink(base, "42", bot_id=3),
                               al.TelegramSink("TOK", "42", base=base))
            assert await g.send("x") and await g.send("y")
            assert [(c[0], c[1]) for c in calls] == [("gw", "post"), ("gw", "patch")]
            state["gw_up"] = False
            calls.clear()
            assert await g.send("z")        # gateway down -> Bot API
            assert [c[0] for c in calls][-1] == "bot"
        finally:
            await srv.close()
    run(go())

    monkeypatch.setenv("TELEGRAM_CHAT_ID", "42")
    monkeypatch.setenv("TELEGRAM_BOT_TOKEN", "t")
    monkeypatch.setenv("TELEGRAM_USE_MCP", "1")
    monkeypatch.setenv("TELEGRAM_MCP_FALLBACK_DIRECT", "0")
    sinks = al.sinks_from_env()
    gw = [s for s in sinks if isinstance(s, al.GatewaySink)][0]
    assert isinstance(gw.primary, al.McpTelegramSink) and gw.fallback is None
    monkeypatch.setenv("TELEGRAM_USE_MCP", "0")
    gw = [s for s in al.sinks_from_env() if isinstance(s, al.GatewaySink)][0]
    assert gw.primary is None and isinstance(gw.fallback, al.TelegramSink)
