"""Alert loop (reference: telemetry/llm_telemetry/main.py:51-220).

Every TELEMETRY_CHECK_INTERVAL (30 s) it takes a snapshot -- job counts,
engine/GPU devices, jobs failed in the last hour with attempts >=
ALERT_FAIL_THRESHOLD -- from the core (``GET /v1/alerts/snapshot``) or
directly from a store.  The first tick is a baseline; later ticks alert on
OFFLINE / ONLINE transitions, a stuck queue (queued > 0, running == 0) and new
failed jobs (ids de-duplicated, at most 100 remembered).  GPU alerts are added
for the MI355X fleet: junction temperature above LMX_ALERT_TEMP_C and a
degraded device circuit.  Sinks: log (always), webhook (ALERT_WEBHOOK_URL),
Telegram Bot API (TELEGRAM_BOT_TOKEN + TELEGRAM_CHAT_ID; edit-in-place, HTML
<pre>, honours 429 retry_after), or a telegram-mcp gateway (TELEGRAM_USE_MCP=1)
with the Bot API as fallback.
"""
from __future__ import annotations

import asyncio
import html
import json
import logging
import os
import time
from datetime import datetime

import aiohttp

log = logging.getLogger("lmx.telemetry")


def snapshot_from_store(store, circuit=None, fail_threshold: int = 3,
                        temp_limit: float = 95.0) -> dict:
    counts = store.job_counts()
    devs = []
    for d in store.list_devices():
        tags = d.get("tags") or {}
        if not (tags.get("engine") or tags.get("ollama") or tags.get("rocm")):
            continue
        devs.append({"id": d["id"], "name": d.get("name") or d["id"],
                     "status": d.get("status"), "temp_c": tags.get("temp_c"),
                     "circuit": circuit.status(d["id"]) if circuit else "ok"})
    failed = [{"id": j["id"], "kind": j["kind"], "error": j.get("error"),
               "attempts": j["attempts"], "max_attempts": j["max_attempts"]}
              for j in store.failed_jobs_since(time.time() - 3600, fail_threshold)][:5]
    return {"queued": counts.get("queued", 0), "running": counts.get("running", 0),
            "devices": devs, "failed_jobs": failed, "temp_limit": temp_limit}


def format_alert(snap: dict, prev_offline: set[str], seen_failed: list[str]) -> str | None:
    lines = []
    offline = {d["id"] for d in snap["devices"] if d["status"] == "offline"}
    names = {d["id"]: d["name"] for d in snap["devices"]}
    for did in sorted(offline - prev_offline):
        lines.append(f"OFFLINE: {names.get(did, did)}")
    for did in sorted(prev_offline - offline):
        lines.append(f"ONLINE: {names.get(did, did)}")
    if snap["queued"] > 0 and snap["running"] == 0:
        lines.append(f"Queue stuck: {snap['queued']} queued, 0 running")
    for d in snap["devices"]:
        t = d.get("temp_c")
        if t is not None and t > snap.get("temp_limit", 95.0):
            lines.append(f"GPU hot: {d['name']} {t:.0f}C")
        if d.get("circuit") == "degraded":
            lines.append(f"Circuit degraded: {d['name']}")
    for j in snap["failed_jobs"]:
        if j["id"] in seen_failed:
            continue
        seen_failed.append(j["id"])
        del seen_failed[:-100]
        err = (j.get("error") or "unknown")[:80]
        lines.append(f"Job failed: {j['kind']} ({j['attempts']}/{j['max_attempts']}) - {err}")
    if not lines:
        return None
    return f"LLM Alert  {datetime.now().astimezone().strftime('%H:%M:%S')}\n" + "\n".join(lines)


class LogSink:
    async def send(self, text: str):
        log.warning("%s", text)
        return True


class WebhookSink:
    def __init__(self, url: str):
        self.url = url

    async def send(self, text: str):
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=10)) as s:
            async with s.post(self.url, json={"text": text}) as r:
                return r.status < 300


def _pre(text: str) -> str:
    return f"<pre>{html.escape(text, quote=False)}</pre>"


class TelegramSink:
    """Direct Bot API client.  The first alert is sent with sendMessage; later
    alerts replace it in place with editMessageText (one live status message
    per chat, reference telemetry/llm_telemetry/telegram_gateway.py:85-101).
    429 answers are retried after ``retry_after``; "message is not modified"
    counts as delivered; an edit of a message that no longer exists falls
    back to a fresh sendMessage."""

    def __init__(self, token: str, chat_id: str, base: str = "https://api.telegram.org"):
        self.url = f"{base}/bot{token}"
        self.chat_id = chat_id
        self.last_id: int | None = None

    async def _call(self, method: str, payload: dict, retries: int = 3):
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=15)) as s:
            for _ in range(retries):
                async with s.post(f"{self.url}/{method}", json=payload) as r:
                    data = await r.json(content_type=None)
                    if r.status == 429:
                        await asyncio.sleep(float((data.get("parameters") or {})
                                                  .get("retry_after", 1)))
                        continue
                    return data
        return {"ok": False}

    async def send_or_edit(self, text: str) -> bool:
        body = {"chat_id": self.chat_id, "text": _pre(text), "parse_mode": "HTML",
                "disable_web_page_preview": True}
        if self.last_id is not None:
            r = await self._call("editMessageText", {**body, "message_id": self.last_id})
            if r.get("ok") or "not modified" in str(r.get("description", "")).lower():
                return True
            self.last_id = None          # deleted / too old to edit: post a new one
        r = await self._call("sendMessage", body)
        if r.get("ok"):
            self.last_id = (r.get("result") or {}).get("message_id")
        return bool(r.get("ok"))

    send = send_or_edit


class McpTelegramSink:
    """Telegram through a telegram-mcp gateway (TELEGRAM_USE_MCP=1,
    reference telegram_gateway.py:104-170): POST {base}/api/messages creates
    the status message, PATCH {base}/api/messages/{id} edits it (the gateway's
    internal id, optional bot_id).  The reference drove the gateway through
    its private telegram_api_client package, which is not available here, so
    the two HTTP routes are this framework's contract (parity unpinned)."""

    def __init__(self, base: str, chat_id: str, bot_id: int | None = None):
        self.base = base.rstrip("/")
        self.chat_id = chat_id
        self.bot_id = bot_id
        self.msg_id: int | None = None

    async def send_or_edit(self, text: str) -> bool:
        body = {"chat_id": self.chat_id, "text": _pre(text), "parse_mode": "HTML",
                "disable_web_page_preview": True}
        if self.bot_id is not None:
            body["bot_id"] = self.bot_id
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=15)) as s:
            if self.msg_id is not None:
                async with s.patch(f"{self.base}/api/messages/{self.msg_id}", json=body) as r:
                    if r.status < 300:
                        return True
                self.msg_id = None
            async with s.post(f"{self.base}/api/messages", json=body) as r:
                if r.status >= 300:
                    return False
                data = await r.json(content_type=None)
        mid = (data or {}).get("id")
        if mid is None:
            return False
        self.msg_id = int(mid)
        return True

    send = send_or_edit


class GatewaySink:
    """Primary route with a fallback (MCP gateway first, direct Bot API when
    it fails and TELEGRAM_MCP_FALLBACK_DIRECT allows, reference
    telemetry/llm_telemetry/main.py:196-211)."""

    def __init__(self, primary, fallback=None):
        self.primary, self.fallback = primary, fallback

    async def send(self, text: str) -> bool:
        ok = False
        if self.primary is not None:
            try:
                ok = await self.primary.send_or_edit(text)
            except Exception as e:
                log.warning("telegram mcp send failed: %s", e)
        if not ok and self.fallback is not None:
            ok = await self.fallback.send_or_edit(text)
        if not ok:
            log.warning("alert send failed (all telegram routes)")
        return ok


def _env_on(name: str, default: bool) -> bool:
    v = os.environ.get(name, "").strip().lower()
    return default if not v else v in ("1", "true", "yes", "y", "on")


def sinks_from_env() -> list:
    s: list = [LogSink()]
    if os.environ.get("ALERT_WEBHOOK_URL"):
        s.append(WebhookSink(os.environ["ALERT_WEBHOOK_URL"]))
    tok = os.environ.get("TELEGRAM_BOT_TOKEN", "").strip()
    chat = (os.environ.get("TELEGRAM_MCP_CHAT_ID") or os.environ.get("TELEGRAM_CHAT_ID")
            or os.environ.get("REPORT_CHAT_ID") or "").strip()
    if not chat:
        return s
    direct = TelegramSink(tok, chat) if tok else None
    if _env_on("TELEGRAM_USE_MCP", False):
        bot = os.environ.get("TELEGRAM_MCP_BOT_ID", "").strip()
        mcp = McpTelegramSink(os.environ.get("TELEGRAM_MCP_BASE_URL", "").strip()
                              or "http://tgapi:8000", chat,
                              int(bot) if bot.lstrip("-").isdigit() else None)
        fb = direct if _env_on("TELEGRAM_MCP_FALLBACK_DIRECT", True) else None
        s.append(GatewaySink(mcp, fb))
    elif direct is not None:
        s.append(GatewaySink(None, direct))
    return s


class AlertLoop:
    def __init__(self, fetch, sinks: list | None = None):
        """fetch: async () -> snapshot dict."""
        self.fetch = fetch
        self.sinks = sinks or [LogSink()]
        self.prev_offline: set[str] | None = None
        self.seen_failed: list[str] = []

    async def tick(self) -> str | None:
        snap = await self.fetch()
        offline = {d["id"] for d in snap["devices"] if d["status"] == "offline"}
        if self.prev_offline is None:  # baseline
            self.prev_offline = offline
            self.seen_failed = [j["id"] for j in snap["failed_jobs"]]
            return None
        text = format_alert(snap, self.prev_offline, self.seen_failed)
        self.prev_offline = offline
        if text:
            for s in self.sinks:
                try:
                    await s.send(text)
                except Exception as e:
                    log.warning("sink %s failed: %s", type(s).__name__, e)
        return text

    async def run(self, interval: float):
        while True:
            try:
                await self.tick()
            except Exception as e:
                log.warning("telemetry tick failed: %s", e)
            await asyncio.sleep(interval)


def http_fetcher(core_url: str):
    async def fetch():
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=10)) as s:
            async with s.get(core_url.rstrip("/") + "/v1/alerts/snapshot") as r:
                return await r.json()
    return fetch


def main():
    logging.basicConfig(level="INFO")
    loop = AlertLoop(http_fetcher(os.environ.get("CORE_HTTP_URL", "http://127.0.0.1:8080")),
                     sinks_from_env())
    asyncio.run(loop.run(float(os.environ.get("TELEMETRY_CHECK_INTERVAL", "30"))))


if __name__ == "__main__":
    main()
