"""Optional cloud chat kinds (openai.chat / openrouter.chat), off the hot path
and disabled unless LMX_ALLOW_CLOUD=1 (reference: worker/llm_worker/main.py:274-327)."""
from __future__ import annotations

import os
import time

import aiohttp


async def cloud_chat(kind: str, payload: dict):
    if os.environ.get("LMX_ALLOW_CLOUD", "0") != "1":
        raise RuntimeError("cloud_disabled")
    prov = kind.split(".")[0]
    if prov == "openai":
        key = os.environ.get("OPENAI_API_KEY", "")
        url = os.environ.get("OPENAI_BASE_URL", "https://api.openai.com/v1") + "/chat/completions"
        model = payload.get("model") or os.environ.get("OPENAI_MODEL", "gpt-4o-mini")
    else:
        key = os.environ.get("OPENROUTER_API_KEY", "")
        url = os.environ.get("OPENROUTER_BASE_URL", "https://openrouter.ai/api/v1").rstrip("/")
        url = url if url.endswith("/chat/completions") else url + "/chat/completions"
        model = payload.get("model") or os.environ.get("OPENROUTER_MODEL", "")
    if not key:
        raise RuntimeError(f"{prov}_api_key_missing")
    body = {"model": model, "messages": payload.get("messages") or
            [{"role": "user", "content": payload.get("prompt", "")}]}
    for k in ("temperature", "max_tokens"):
        if payload.get(k) is not None:
            body[k] = payload[k]
    t0 = time.time()
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=120)) as s:
        async with s.post(url, json=body, headers={"Authorization": f"Bearer {key}"}) as r:
            if r.status >= 400:
                raise RuntimeError(f"{prov} HTTP {r.status}: {(await r.text())[:300]}")
            data = await r.json()
    ms = int((time.time() - t0) * 1000)
    usage = data.get("usage") or {}
    tin, tout = int(usage.get("prompt_tokens", 0)), int(usage.get("completion_tokens", 0))
    msg = ((data.get("choices") or [{}])[0].get("message") or {})
    from .jobs import calc_cost
    res = {"ok": True, "response": msg.get("content", ""), "model": data.get("model", model),
           "provider": prov, "tier": payload.get("_tier", ""), "tokens_in": tin,
           "tokens_out": tout, "cost": calc_cost(payload, tin, tout), "data": data}
    if msg.get("reasoning") and payload.get("thinking", True):
        res["thinking"] = msg["reasoning"]
    return res, {"ms": ms, "model": res["model"], "provider": prov, "tokens_in": tin,
                 "tokens_out": tout}
