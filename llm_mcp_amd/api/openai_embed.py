"""``POST /v1/embeddings`` -- OpenAI-compatible, served by the in-process
encoder on a local GPU (reference: core/internal/api/handlers.go:1821-2078).

Kept: ``input`` string|[]string -> texts (400 invalid_input / empty_input),
``model`` required, cloud ids (with ``/``) go to OpenRouter only when cloud is
enabled (client-side Matryoshka truncation with CLOUD_EMBED_DIMENSIONS), local
ids get up to 3 attempts over healthy replicas with the circuit breaker fed
on every outcome, 503 ``no_device`` when no replica exists, 502
``embed_failed`` when all attempts fail, OpenAI list response with usage.
Extended: ``dimensions`` applies to local models too (truncate + re-normalise
on the GPU), ``encoding_format: base64``, token-id inputs.
"""
from __future__ import annotations

import asyncio
import base64
import json
import os
import time

import numpy as np
from aiohttp import web

from ..native import runtime
from .helpers import read_json, write_error

EMBED_TIMEOUT_S = 120.0


def _texts(inp):
    if isinstance(inp, str):
        return [inp], None
    if isinstance(inp, list):
        if inp and all(isinstance(x, int) for x in inp):
            return None, [inp]
        if inp and all(isinstance(x, list) for x in inp):
            return None, [[int(t) for t in x] for x in inp]
        return [x for x in inp if isinstance(x, str)], None
    return None, None


def _response(vecs, fmt: str, model: str, ntok: int) -> web.Response:
    """OpenAI list response.  The float form is spliced from rows formatted
    natively (``_lmx_runtime.f32_json_rows``: shortest float32 round-trip
    text); json.dumps over Python floats costs ~7 ms per 16 x 768 response
    and bounded the API process."""
    arr = np.asarray(vecs, dtype=np.float32).reshape(len(vecs), -1)
    if fmt == "base64":
        rows = ['"' + base64.b64encode(arr[i].astype("<f4").tobytes()).decode() + '"'
                for i in range(len(arr))]
    else:
        rows = runtime().f32_json_rows(arr)
    data = ",".join('{"object":"embedding","embedding":%s,"index":%d}' % (r, i)
                    for i, r in enumerate(rows))
    body = '{"object":"list","data":[%s],"model":%s,"usage":{"prompt_tokens":%d,' \
           '"total_tokens":%d}}\n' % (data, json.dumps(model, ensure_ascii=False), ntok, ntok)
    return web.Response(status=200, text=body, content_type="application/json")


class EmbeddingsHandler:
    def __init__(self, state):
        self.state = state

    async def __call__(self, request):
        st = self.state
        if request.method != "POST":
            return write_error(405, "method_not_allowed", "Only POST allowed")
        try:
            body = await read_json(request)
        except ValueError:
            return write_error(400, "invalid_json", "Invalid JSON body")
        if not isinstance(body, dict):
            return write_error(400, "invalid_json", "Invalid JSON body")
        model = body.get("model") or ""
        if not model:
            return write_error(400, "model_required", "Field 'model' is required")
        texts, token_ids = _texts(body.get("input"))
        if texts is None and token_ids is None:
            return write_error(400, "invalid_input",
                               "Field 'input' must be a string or array of strings")
        if texts is not None and not texts:
            return write_error(400, "empty_input", "Input is empty")
        dims = body.get("dimensions")
        dims = int(dims) if isinstance(dims, (int, float)) and int(dims) > 0 else None
        fmt = body.get("encoding_format") or "float"
        if "/" in model:
            cloud = getattr(st, "cloud_embed", None)
            if cloud is None:
                return write_error(503, "cloud_disabled",
                                   "Cloud models are disabled (LMX_ALLOW_CLOUD=1 and "
                                   "OPENROUTER_API_KEY)")
            return await cloud(body, model, texts, dims or int(os.environ.get(
                "CLOUD_EMBED_DIMENSIONS", "0") or 0))
        last_err = None
        tried = set()
        for attempt in range(3):
            target = st.registry.select(model, "embed", getattr(st, "circuit", None))
            if target is not None and target.device_id in tried:
                others = [m for m in st.registry.replicas(model)
                          if m.kind == "embed" and m.device_id not in tried]
                target = others[0] if others else target
            if target is None:
                if attempt == 0:
                    st.metrics.embedding_requests.labels(model, "none", "no_device").inc()
                    return write_error(503, "no_device", f"No online device has model '{model}'")
                break
            tried.add(target.device_id)
            t0 = time.time()
            try:
                seqs = token_ids if token_ids is not None else [
                    target.tokenizer.encode(t, add_bos=True) + list(target.tokenizer.eos_ids[:1])
                    for t in texts]
                if dims and dims > target.cfg.embed_dim:
                    return write_error(400, "invalid_dimensions",
                                       f"dimensions must be <= {target.cfg.embed_dim}")
                st.registry.acquire(target)
                try:
                    vecs = await asyncio.wait_for(target.engine.embed(seqs, dims),
                                                  EMBED_TIMEOUT_S)
                finally:
                    st.registry.release(target)
            except Exception as e:  # device failure: circuit + retry elsewhere
                last_err = e
                st.circuit.record(target.device_id, False)
                continue
            el = time.time() - t0
            st.circuit.record(target.device_id, True)
            ntok = sum(len(s) for s in seqs)
            m = st.metrics
            m.embedding_requests.labels(model, target.device_id, "ok").inc()
            m.embedding_duration.labels(model, target.device_id).observe(el)
            m.embedding_tokens.labels(model, target.device_id).inc(ntok)
            return _response(vecs, fmt, model, ntok)
        st.metrics.embedding_requests.labels(model, "all", "error").inc()
        return write_error(502, "embed_failed", str(last_err) if last_err else
                           "All devices failed")
