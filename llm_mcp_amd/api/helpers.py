"""HTTP helpers: JSON writer, the reference's error contract
``{error, message, details}`` (core/internal/models/types.go:14-18,
core/internal/api/helpers.go:11-29), SSE framing and number coercion."""
from __future__ import annotations

import json

from aiohttp import web


def dumps(obj) -> str:
    return json.dumps(obj, separators=(",", ":"), ensure_ascii=False, default=str)


def write_json(status: int, payload) -> web.Response:
    return web.Response(status=status, text=dumps(payload) + "\n",
                        content_type="application/json")


def write_error(status: int, code: str, message: str = "", details: str = "") -> web.Response:
    body = {"error": code}
    if message:
        body["message"] = message
    if details:
        body["details"] = details
    return write_json(status, body)


def sse_frame(event: str | None, payload) -> bytes:
    data = payload if isinstance(payload, str) else dumps(payload)
    head = f"event: {event}\n" if event else ""
    return f"{head}data: {data}\n\n".encode()


def to_int(v, default: int | None = None):
    if isinstance(v, bool):
        return default
    if isinstance(v, (int, float)):
        return int(v)
    if isinstance(v, str):
        try:
            return int(float(v))
        except ValueError:
            return default
    return default


def method_guard(request: web.Request, allowed: str) -> web.Response | None:
    if request.method != allowed:
        return write_error(405, "method_not_allowed", f"Only {allowed} allowed")
    return None


async def read_json(request: web.Request, limit: int = 10 << 20):
    raw = await request.content.read(limit + 1)
    if len(raw) > limit:
        raise ValueError("body_too_large")
    if not raw.strip():
        return {}
    return json.loads(raw)
