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
<pre>, honours 429 retry_after).
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


class TelegramSink:
    """Direct Bot API client (edit-in-place of the last alert message)."""

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

    async def send(self, text: str):
        body = {"chat_id": self.chat_id, "text": f"<pre>{html.escape(text)}</pre>",
                "parse_mode": "HTML"}
        r = await self._call("sendMessage", body)
        if r.get("ok"):
            self.last_id = (r.get("result") or {}).get("message_id")
        return bool(r.get("ok"))


def sinks_from_env() -> list:
    s: list = [LogSink()]
    if os.environ.get("ALERT_WEBHOOK_URL"):
        s.append(WebhookSink(os.environ["ALERT_WEBHOOK_URL"]))
    tok = os.environ.get("TELEGRAM_BOT_TOKEN")
    chat = os.environ.get("TELEGRAM_CHAT_ID") or os.environ.get("REPORT_CHAT_ID")
    if tok and chat:
        s.append(TelegramSink(tok, chat))
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
