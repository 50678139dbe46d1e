"""Request IDs and per-request spans.

The reference has no request correlation: timing is ad hoc ``time.Since`` in
the Go handlers (core/internal/api/handlers.go:1878-1880,2164,2222) and
``perf_counter`` ms in the worker (worker/llm_worker/main.py:238-240), with no
ID tying an HTTP request to the job row, the worker attempt or the engine.

Here one request ID follows a request through every hop:

* HTTP: ``X-Request-ID`` is honoured from the client or minted by the
  middleware, set on a context var for the handler and echoed on the
  response;
* store: a job submitted with a client ``X-Request-ID`` carries it as
  ``payload._request_id`` (the reference's convention for internal payload
  fields, cf. ``_tier`` / ``_price_in_1m``); without one the job ID is the
  correlation key, so stored payloads stay exactly as submitted;
* worker: the attempt's span (queue wait, run, TTFT, tokens) is tagged with
  it and its ID is returned in the completion metrics;
* chat: the sync/stream path records TTFT (queue + prefill), decode and total.

Spans are logged as one JSON line each on the ``llm_mcp_amd.trace`` logger
and kept in a bounded in-memory ring (``GET /v1/debug/trace/{request_id}``).
"""
from __future__ import annotations

import collections
import contextvars
import json
import logging
import threading
import time
import uuid

HEADER = "X-Request-ID"
PAYLOAD_KEY = "_request_id"
MAX_ID_LEN = 128

log = logging.getLogger("llm_mcp_amd.trace")
current_request_id: contextvars.ContextVar[str] = contextvars.ContextVar(
    "lmx_request_id", default="")


def new_id() -> str:
    return uuid.uuid4().hex


def clean_id(rid) -> str:
    """A client-supplied ID is kept if it is short printable ASCII, else
    dropped (IDs end up in logs and headers)."""
    if not isinstance(rid, str):
        return ""
    rid = rid.strip()
    if not rid or len(rid) > MAX_ID_LEN or not rid.isascii() or not rid.isprintable():
        return ""
    return rid


class SpanRing:
    """Last ``maxlen`` spans, searchable by request ID (thread-safe: worker
    threads and the event loop both record)."""

    def __init__(self, maxlen: int = 4096):
        self._lock = threading.Lock()
        self._spans: collections.deque = collections.deque(maxlen=maxlen)

    def add(self, span: dict) -> None:
        with self._lock:
            self._spans.append(span)

    def find(self, request_id: str) -> list[dict]:
        with self._lock:
            return [dict(s) for s in self._spans if s.get("request_id") == request_id]

    def clear(self) -> None:
        with self._lock:
            self._spans.clear()


RING = SpanRing()


def record_span(name: str, request_id: str, **fields) -> dict:
    """Record one span: ``name`` (``chat``, ``job.attempt``, ...), the request
    ID and its fields (durations in ms; ``None`` fields are dropped)."""
    span = {"span": name, "request_id": request_id or "", "ts": round(time.time(), 6)}
    for k, v in fields.items():
        if v is None:
            continue
        span[k] = round(v, 3) if isinstance(v, float) else v
    RING.add(span)
    if log.isEnabledFor(logging.INFO):
        log.info(json.dumps(span, separators=(",", ":")))
    return span


def tag_payload(payload: dict, request_id: str) -> dict:
    """Copy of a job payload carrying the request ID (an ID already in the
    payload wins: a resubmitted job keeps its original correlation)."""
    if not request_id or clean_id(payload.get(PAYLOAD_KEY)):
        return payload
    out = dict(payload)
    out[PAYLOAD_KEY] = request_id
    return out


def payload_request_id(payload) -> str:
    if isinstance(payload, dict):
        return clean_id(payload.get(PAYLOAD_KEY))
    return ""


def client_request_id(request) -> str:
    """The ID the client sent (empty when the middleware minted one)."""
    return clean_id(request.headers.get(HEADER))


def aiohttp_middleware():
    """aiohttp middleware: request ID in, on the ``current_request_id``
    context var for the handler, echoed on the response (streaming handlers pass it in
    their headers before ``prepare``; a prepared response is left alone)."""
    from aiohttp import web

    @web.middleware
    async def request_id_mw(request, handler):
        rid = clean_id(request.headers.get(HEADER)) or new_id()
        tok = current_request_id.set(rid)
        try:
            resp = await handler(request)
        except web.HTTPException as e:
            e.headers.setdefault(HEADER, rid)
            raise
        finally:
            current_request_id.reset(tok)
        if not resp.prepared:
            resp.headers.setdefault(HEADER, rid)
        return resp

    return request_id_mw
