"""Batched embedding engine (one per GPU that serves an embedding model).

Requests (each a list of token-id sequences) queue up; the engine thread packs
as many whole requests as fit ``max_batch_tokens`` into one varlen forward of
the encoder, so concurrent /v1/embeddings calls share GEMMs (the reference
made one Ollama HTTP call per request, core/internal/api/handlers.go:1942).
Results are delivered to asyncio futures with one call_soon_threadsafe per
batch."""
from __future__ import annotations

import asyncio
import logging
import os
import queue
import threading
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..models.bert import BertModel
from ..models.config import BertConfig, NomicBertConfig
from ..models.nomic_bert import NomicBertModel

log = logging.getLogger("lmx.embed")


@dataclass
class EmbedRequest:
    seqs: list[list[int]]
    dims: int | None
    future: object = None
    loop: object = None
    result: list | None = None
    error: str | None = None
    done: threading.Event = field(default_factory=threading.Event)


class EmbeddingEngine:
    def __init__(self, cfg: NomicBertConfig | BertConfig, device="cuda",
                 max_batch_tokens: int | None = None, max_seq_len: int = 2048, seed: int = 0,
                 weights=None):
        # 64k tokens per forward: the K13 encoder GEMMs and the attention fill
        # the chip better than at 32k (nomic, 1k-token docs: 2,927 vs 2,882
        # emb/s, profiles/r6_serving/embed_batch.log)
        if max_batch_tokens is None:
            max_batch_tokens = int(os.environ.get("LMX_EMBED_BATCH_TOKENS", "65536"))
        self.cfg = cfg
        self.device = torch.device(device)
        model_cls = BertModel if isinstance(cfg, BertConfig) else NomicBertModel
        self.model = model_cls(cfg, self.device, seed=seed, weights=weights)
        self.max_batch_tokens = max_batch_tokens
        self.max_seq_len = min(max_seq_len, cfg.max_position)
        self._q: queue.SimpleQueue = queue.SimpleQueue()
        self._stop = threading.Event()
        self._thread = None
        self.stats = {"batches": 0, "sequences": 0, "tokens": 0, "time_s": 0.0}

    def start(self):
        if self._thread is None:
            self._stop.clear()
            self._thread = threading.Thread(target=self._loop, daemon=True, name="lmx-embed")
            self._thread.start()

    def stop(self):
        self._stop.set()
        self._q.put(None)
        if self._thread is not None:
            self._thread.join(timeout=10)
            self._thread = None

    def _truncate(self, seqs):
        return [s[: self.max_seq_len] if len(s) else [0] for s in seqs]

    # synchronous API (worker jobs, tests)
    def embed_sync(self, seqs: list[list[int]], dims: int | None = None) -> list[list[float]]:
        return self._run([EmbedRequest(self._truncate(seqs), dims)])[0]

    # asyncio API
    async def embed(self, seqs: list[list[int]], dims: int | None = None) -> list[list[float]]:
        loop = asyncio.get_running_loop()
        req = EmbedRequest(self._truncate(seqs), dims, loop.create_future(), loop)
        self._q.put(req)
        return await req.future

    def _loop(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        pending: list[EmbedRequest] = []
        inflight = None
        while not self._stop.is_set():
            if not pending and inflight is None:
                item = self._q.get()
                if item is None:
                    break
                pending.append(item)
            while True:  # drain whatever else is waiting
                try:
                    item = self._q.get_nowait()
                except queue.Empty:
                    break
                if item is None:
                    self._stop.set()
                    break
                pending.append(item)
            batch, ntok = [], 0
            while pending:
                n = sum(len(s) for s in pending[0].seqs)
                if batch and ntok + n > self.max_batch_tokens:
                    break
                batch.append(pending.pop(0))
                ntok += n
            # two batches in flight: batch n+1's host prep and launch overlap
            # batch n's kernels; batch n is finished (synced) afterwards
            launched = None
            if batch:
                try:
                    launched = self._launch(batch)
                except Exception as e:
                    log.exception("embedding batch failed")
                    for r in batch:
                        self._deliver(r, None, str(e))
            if inflight is not None:
                self._complete(inflight)
            inflight = launched
            if inflight is not None and not pending and self._q.empty():
                self._complete(inflight)
                inflight = None
        if inflight is not None:
            self._complete(inflight)

    def _complete(self, launched):
        batch = launched[0]
        try:
            outs = self._finish(launched)
            for r, o in zip(batch, outs):
                self._deliver(r, o, None)
        except Exception as e:
            log.exception("embedding batch failed")
            for r in batch:
                self._deliver(r, None, str(e))

    @staticmethod
    def _deliver(r: EmbedRequest, out, err):
        r.result, r.error = out, err
        r.done.set()
        if r.future is not None:
            def _set(f=r.future):
                if f.done():
                    return
                if err is None:
                    f.set_result(out)
                else:
                    f.set_exception(RuntimeError(err))
            r.loop.call_soon_threadsafe(_set)

    def _run(self, batch: list[EmbedRequest]) -> list[list[list[float]]]:
        return self._finish(self._launch(batch))

    @torch.no_grad()
    def _launch(self, batch: list[EmbedRequest]):
        """Queue one varlen encoder forward; returns the pending result."""
        t0 = time.perf_counter()
        seqs = [s for r in batch for s in r.seqs]
        lens = [len(s) for s in seqs]
        flat = np.concatenate([np.asarray(s, dtype=np.int32) for s in seqs])
        cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
        ids = torch.from_numpy(flat).to(self.device, non_blocking=True)
        cu_t = torch.from_numpy(cu).to(self.device, non_blocking=True)
        dims = {r.dims or self.cfg.embed_dim for r in batch}
        fused = len(dims) == 1
        if fused:
            # pooling, Matryoshka truncation and L2 norm fused in one kernel (K9)
            dev_out = self.model.forward(ids, cu_t, lens, dims=dims.pop(), normalize=True)
        else:
            dev_out = self.model.forward(ids, cu_t, lens, dims=None, normalize=False)
        if self.device.type == "cuda":
            host = torch.empty(dev_out.shape, dtype=dev_out.dtype, pin_memory=True)
            host.copy_(dev_out, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = dev_out, None
        return batch, host, ev, fused, len(flat), t0

    def _finish(self, launched) -> list[list[list[float]]]:
        batch, full, ev, fused, ntok, t0 = launched
        if ev is not None:
            ev.synchronize()
        outs, k = [], 0
        for r in batch:
            e = full[k:k + len(r.seqs)]
            k += len(r.seqs)
            if not fused:
                e = e[:, :r.dims or self.cfg.embed_dim]
                e = e / e.norm(dim=-1, keepdim=True).clamp_min(1e-12)
            # float32 rows (consumers needing JSON lists call .tolist(); the
            # engine socket ships the bytes)
            outs.append(e.float().numpy())
        self.stats["batches"] += 1
        self.stats["sequences"] += sum(len(r.seqs) for r in batch)
        self.stats["tokens"] += ntok
        self.stats["time_s"] += time.perf_counter() - t0
        return outs
