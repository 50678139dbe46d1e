"""asyncio front of an engine: per-request async token streams.

The engine thread hands over one batched event list per step; a single
``call_soon_threadsafe`` per step fans it out to the per-request queues, so
the event loop is woken once per step regardless of the batch size.  This is
the in-process replacement of the reference's core -> Ollama NDJSON stream
(core/internal/api/handlers.go:2505-2573)."""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field
from typing import AsyncIterator

from .engine import GenRequest, SamplingParams, TokenEvent


@dataclass
class StreamItem:
    token: int
    logprob: float
    finish: str | None


@dataclass
class RequestStats:
    arrival: float = 0.0
    first_token: float = 0.0
    last_token: float = 0.0
    prompt_tokens: int = 0
    completion_tokens: int = 0
    finish: str | None = None
    token_times: list[float] = field(default_factory=list)


class AsyncEngine:
    """Wraps an LLMEngine (or any object with submit/abort/start/stop and an
    ``event_sink`` attribute)."""

    def __init__(self, engine, loop: asyncio.AbstractEventLoop | None = None):
        self.engine = engine
        self.loop = loop
        self._queues: dict[int, asyncio.Queue] = {}
        engine.event_sink = self._sink

    def start(self, loop: asyncio.AbstractEventLoop | None = None):
        self.loop = loop or self.loop or asyncio.get_event_loop()
        self.engine.start()

    def stop(self):
        self.engine.stop()

    # engine thread
    def _sink(self, evs: list[TokenEvent]):
        loop = self.loop
        if loop is None or loop.is_closed():
            return
        loop.call_soon_threadsafe(self._dispatch, evs)

    # event loop
    def _dispatch(self, evs: list[TokenEvent]):
        for e in evs:
            q = self._queues.get(e.req.id)
            if q is not None:
                q.put_nowait(StreamItem(e.token, e.logprob, e.finish))

    async def generate(self, prompt_ids: list[int], params: SamplingParams, priority: int = 0,
                       stats: RequestStats | None = None) -> AsyncIterator[StreamItem]:
        """Yields StreamItems; the last one carries ``finish``.  Cancelling the
        consumer aborts the request in the engine."""
        req = GenRequest(list(prompt_ids), params, priority=priority)
        req.id = next(self.engine._ids)
        q: asyncio.Queue = asyncio.Queue()
        self._queues[req.id] = q
        if stats is not None:
            stats.arrival = time.time()
            stats.prompt_tokens = len(prompt_ids)
        self.engine.submit(req)
        done = False
        try:
            while True:
                item: StreamItem = await q.get()
                if stats is not None and item.token >= 0:
                    now = time.time()
                    if not stats.first_token:
                        stats.first_token = now
                    stats.last_token = now
                    stats.completion_tokens += 1
                yield item
                if item.finish is not None:
                    done = True
                    if stats is not None:
                        stats.finish = item.finish
                    return
        finally:
            self._queues.pop(req.id, None)
            if not done:
                self.engine.abort(req.id)

    async def complete(self, prompt_ids, params, priority=0):
        toks, lps, fin = [], [], None
        async for it in self.generate(prompt_ids, params, priority):
            if it.token >= 0:
                toks.append(it.token)
                lps.append(it.logprob)
            fin = it.finish
        return toks, lps, fin
