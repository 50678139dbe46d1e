"""``POST /v1/chat/completions`` -- OpenAI-compatible, sync and SSE stream,
served by the in-process engine of the selected GPU.

Contract kept from the reference (core/internal/api/handlers.go:2087-2587):
  * 10 MB body cap, ``messages`` required (400 ``messages_required``);
  * empty ``model`` -> smart selection from headers ``X-Task-Type`` /
    ``X-Accuracy`` / ``X-Max-Cost`` (response header ``X-Selected-Model``);
  * model ids containing ``/`` are cloud models: proxied to OpenRouter only
    when ``LMX_ALLOW_CLOUD=1`` (the hot path never falls back to the cloud);
  * stream frames: ``data: {chat.completion.chunk}\\n\\n`` ... a final chunk
    with empty delta and ``finish_reason``, then ``data: [DONE]\\n\\n``;
  * non-stream: ``chat.completion`` with ``usage``.
Defect fixed: ``max_tokens``, ``top_p`` and ``stop`` are honoured (the
reference parsed and dropped them, handlers.go:2333-2340); ``top_k``,
``seed``, ``logprobs``, ``stream_options.include_usage`` and the OpenAI
``presence_penalty`` / ``frequency_penalty`` (plus ``repetition_penalty`` and
Ollama's ``options.repeat_penalty`` / ``repeat_last_n``) are supported.
"""
from __future__ import annotations

import json
import logging
import time
import uuid

from aiohttp import web

from ..engine.async_engine import StreamItem
from ..engine.engine import SamplingParams
from ..models.tokenizer import IncrementalDetokenizer, apply_chat_template
from ..utils import tracing
from .helpers import dumps, read_json, write_error, write_json

log = logging.getLogger("lmx.chat")
RESTART = StreamItem(-2, 0.0, None)   # _failover: generation restarted on another replica

CHAT_TIMEOUT_S = 120.0


def sampling_from_body(body: dict, max_len_left: int) -> SamplingParams:
    def f(name, default):
        v = body.get(name)
        return default if v is None else v

    stop = body.get("stop")
    if isinstance(stop, str):
        stop = [stop]
    elif not isinstance(stop, list):
        stop = []
    max_tokens = body.get("max_tokens", body.get("max_completion_tokens"))
    if max_tokens is None:
        max_tokens = min(max_len_left, 1024)
    opts = body.get("options") or {}  # Ollama-style options also accepted
    return SamplingParams(
        temperature=float(f("temperature", opts.get("temperature", 0.8))),
        top_p=float(f("top_p", opts.get("top_p", 1.0))),
        top_k=int(f("top_k", opts.get("top_k", 0))),
        max_tokens=max(1, min(int(max_tokens), max_len_left)),
        stop=[str(s) for s in stop][:16],
        ignore_eos=bool(body.get("ignore_eos", False)),
        seed=body.get("seed", opts.get("seed")),
        logprobs=bool(body.get("logprobs", False)),
        presence_penalty=float(f("presence_penalty", opts.get("presence_penalty", 0.0))),
        frequency_penalty=float(f("frequency_penalty", opts.get("frequency_penalty", 0.0))),
        repetition_penalty=float(f("repetition_penalty", opts.get("repeat_penalty", 1.0))),
        penalty_last_n=penalty_window(opts.get("repeat_last_n", 64)))


def penalty_window(n) -> int:
    """Ollama repeat_last_n: -1 = whole context (capped at the kernel's 64-token
    window), 0 = off."""
    n = int(n)
    return 64 if n < 0 else min(n, 64)


def logprob_item(tok, token: int, logprob: float, as_ids: bool = False) -> dict:
    """One OpenAI ``logprobs.content`` entry: the token's text (or
    ``token_id:<id>`` with ``return_tokens_as_token_ids``), its logprob and
    its UTF-8 bytes (the sampler reports the chosen token only: no
    top_logprobs alternatives)."""
    b = tok.token_bytes(token)
    return {"token": f"token_id:{token}" if as_ids else b.decode("utf-8", errors="replace"),
            "logprob": logprob, "bytes": list(b), "top_logprobs": []}


class ChatHandler:
    def __init__(self, state):
        self.state = state

    async def __call__(self, request: web.Request) -> web.StreamResponse:
        st = self.state
        if request.method != "POST":
            return write_error(405, "method_not_allowed", "Only POST allowed")
        try:
            body = await read_json(request)
        except ValueError as e:
            if str(e) == "body_too_large":
                return write_error(413, "body_too_large", "Request body exceeds 10MB")
            return write_error(400, "invalid_json", "Invalid JSON body")
        if not isinstance(body, dict):
            return write_error(400, "invalid_json", "Invalid JSON body")
        messages = body.get("messages")
        if not isinstance(messages, list) or not messages:
            return write_error(400, "messages_required", "Field 'messages' is required")
        model = body.get("model") or ""
        # request id: honoured from the client or minted here,
        # echoed on the response and logged with the completion record
        rid = tracing.current_request_id.get() or tracing.clean_id(
            request.headers.get(tracing.HEADER)) or tracing.new_id()
        extra_headers = {tracing.HEADER: rid}
        if not model:
            selector = getattr(st, "select_model", None)
            selected = None
            if selector is not None:
                selected = await selector(request, body)
            if not selected:
                return write_error(400, "no_model", "Could not select a model. Specify 'model' "
                                   "explicitly or seed model_rankings.")
            model = selected
            extra_headers["X-Selected-Model"] = model
        if "/" in model:
            cloud = getattr(st, "cloud_chat", None)
            if cloud is None:
                return write_error(503, "cloud_disabled",
                                   "Cloud models are disabled (set LMX_ALLOW_CLOUD=1 and "
                                   "OPENROUTER_API_KEY)")
            return await cloud(request, body, model, extra_headers)
        # the replica that serves the request, counted against the node-wide
        # load in the same step as its selection (failover moves it); one
        # selection per request: a validation error below releases it
        target = st.registry.select(model, "chat", getattr(st, "circuit", None), acquire=True)
        if target is None:
            st.metrics.chat_requests(model, "none", "no_device")
            return write_error(503, "no_device", f"No online device has model '{model}'")
        box = {"target": target}
        try:
            tok = target.tokenizer
            try:
                prompt_ids = apply_chat_template(tok, messages)
            except Exception as e:
                return write_error(400, "invalid_messages", str(e))
            left = target.max_model_len - len(prompt_ids) - 1
            if left < 1:
                return write_error(400, "context_length_exceeded",
                                   f"prompt has {len(prompt_ids)} tokens; model context is "
                                   f"{target.max_model_len}")
            params = sampling_from_body(body, left)
            stream = bool(body.get("stream", False))
            include_usage = bool((body.get("stream_options") or {}).get("include_usage", False))
            n = body.get("n")
            try:
                n = 1 if n is None else int(n)
            except (TypeError, ValueError):
                n = 0
            if not 1 <= n <= 16:
                return write_error(400, "invalid_n", "'n' must be an integer in [1, 16]")
            # vLLM's extension: logprobs entries name their token as "token_id:<id>"
            box["ids"] = bool(body.get("return_tokens_as_token_ids", False))
            t0 = time.time()
            if n > 1:
                return await self._multi(request, target, model, prompt_ids, params, n, stream,
                                         include_usage, extra_headers, t0, box["ids"])
            if stream:
                return await self._stream(request, box, model, prompt_ids, params,
                                          include_usage, extra_headers, t0)
            return await self._sync(box, model, prompt_ids, params, extra_headers, t0)
        finally:
            st.registry.release(box["target"])

    async def _failover(self, box, model, prompt_ids, params, attempts: int = 3,
                        restartable: bool = False):
        """The engine's token stream, moved to another healthy replica when
        the serving engine fails BEFORE its first token (worker died, HIP
        fault): nothing reached the client yet, so the request is simply
        resubmitted (up to ``attempts`` replicas).  ``restartable`` (the
        non-streaming response, buffered until the end): a failure after
        tokens also moves the request; a ``RESTART`` item tells the caller to
        drop what it collected.  After a streamed token the error is the
        client's, as in the reference."""
        st = self.state
        circuit = getattr(st, "circuit", None)
        tried = {box["target"].device_id}
        while True:
            gen = box["target"].engine.generate(prompt_ids, params)
            emitted, failed = False, None
            try:
                async for it in gen:
                    if it.token >= 0:
                        emitted = True
                    if (it.finish is not None and it.finish.startswith("error")
                            and (restartable or not emitted)):
                        failed = it
                        break
                    yield it
                    if it.finish is not None:
                        return
            except ConnectionError as e:          # link already down at submit
                if emitted and not restartable:
                    raise
                failed = StreamItem(-1, 0.0, f"error:{e}")
            finally:
                await gen.aclose()
            if failed is None:
                return
            if circuit is not None:
                circuit.record(box["target"].device_id, False)
            nxt = None if len(tried) >= attempts else \
                st.registry.select(model, "chat", circuit, exclude=tried, acquire=True)
            if nxt is None:
                yield failed
                return
            log.warning("chat request failed on %s before its first token (%s); retrying on %s",
                        box["target"].device_id, failed.finish, nxt.device_id)
            st.registry.release(box["target"])
            box["target"] = nxt
            tried.add(nxt.device_id)
            if emitted:
                yield RESTART

    async def _multi(self, request, target, model, prompt_ids, params, n, stream, include_usage,
                     headers, t0, as_ids=False):
        """``n`` choices: n engine requests of the same prompt (seeds seed+i, or
        distinct per-request seeds), batched by the engine like any other
        concurrent requests; streamed chunks carry their choice ``index``."""
        import asyncio
        import dataclasses
        base = params.seed if params.seed is not None else uuid.uuid4().int & 0x7FFFFFFF
        plist = [dataclasses.replace(params, seed=base + i) for i in range(n)]
        q: asyncio.Queue = asyncio.Queue()
        stats = {"ttft": None, "n_out": 0, "errors": 0}

        async def run(i, sp):
            detok = IncrementalDetokenizer(target.tokenizer, sp.stop)
            finish, lps = "stop", []
            gen = target.engine.generate(prompt_ids, sp)
            try:
                async for it in gen:
                    if it.token >= 0:
                        stats["n_out"] += 1
                        if stats["ttft"] is None:
                            stats["ttft"] = time.time() - t0
                        piece = detok.push(it.token)
                        lp = logprob_item(target.tokenizer, it.token, it.logprob, as_ids) \
                            if sp.logprobs else None
                        await q.put((i, piece, None, lp))
                        if detok.stopped:
                            break
                    if it.finish is not None:
                        finish = it.finish
                        break
            finally:
                await gen.aclose()
            tail = detok.flush()
            if finish.startswith("error"):
                stats["errors"] += 1
                finish = "error"
            elif finish not in ("stop", "length"):
                finish = "stop"
            await q.put((i, tail, finish, None))

        tasks = [asyncio.ensure_future(run(i, sp)) for i, sp in enumerate(plist)]
        chat_id = "chatcmpl-" + uuid.uuid4().hex[:24]
        created = int(time.time())
        status = "ok"
        try:
            if not stream:
                texts, fins, lps = [[] for _ in range(n)], [None] * n, [[] for _ in range(n)]
                left = n
                while left:
                    i, piece, fin, lp = await q.get()
                    texts[i].append(piece)
                    if fin is not None:
                        fins[i] = fin
                        left -= 1
                    elif lp is not None and params.logprobs:
                        lps[i].append(lp)
                if stats["errors"]:
                    status = "error"
                    return write_error(502, "engine_failed", "a choice failed in the engine")
                choices = []
                for i in range(n):
                    c = {"index": i, "message": {"role": "assistant", "content": "".join(texts[i])},
                         "finish_reason": fins[i]}
                    if params.logprobs:
                        c["logprobs"] = {"content": lps[i]}
                    choices.append(c)
                resp = {"id": chat_id, "object": "chat.completion", "created": created,
                        "model": model, "choices": choices,
                        "usage": {"prompt_tokens": len(prompt_ids),
                                  "completion_tokens": stats["n_out"],
                                  "total_tokens": len(prompt_ids) + stats["n_out"]}}
                r = write_json(200, resp)
                r.headers.update(headers)
                return r
            resp = web.StreamResponse(status=200, headers={
                "Content-Type": "text/event-stream", "Cache-Control": "no-cache",
                "Connection": "keep-alive", **headers})
            await resp.prepare(request)
            started = [False] * n
            left = n

            def chunk(i, delta, fin=None, lp=None):
                c = {"index": i, "delta": delta, "finish_reason": fin}
                if lp is not None:
                    c["logprobs"] = {"content": [lp]}
                return b"data: " + dumps({"id": chat_id, "object": "chat.completion.chunk",
                                          "created": created, "model": model,
                                          "choices": [c]}).encode() + b"\n\n"
            try:
                while left:
                    i, piece, fin, lp = await q.get()
                    if piece or not started[i] or lp is not None:
                        delta = {"content": piece}
                        if not started[i]:
                            delta["role"] = "assistant"
                            started[i] = True
                        await resp.write(chunk(i, delta, lp=lp))
                    if fin is not None:
                        left -= 1
                        await resp.write(chunk(i, {}, fin))
                if stats["errors"]:
                    status = "error"
                if include_usage:
                    await resp.write(b"data: " + dumps({
                        "id": chat_id, "object": "chat.completion.chunk", "created": created,
                        "model": model, "choices": [],
                        "usage": {"prompt_tokens": len(prompt_ids),
                                  "completion_tokens": stats["n_out"],
                                  "total_tokens": len(prompt_ids) + stats["n_out"]}}).encode()
                        + b"\n\n")
                await resp.write(b"data: [DONE]\n\n")
            except (ConnectionResetError, ConnectionError):
                status = "client_gone"
            return resp
        finally:
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
            self._record(target, model, status, t0, len(prompt_ids), stats["n_out"],
                         stats["ttft"], headers.get(tracing.HEADER, ""), n=n)

    async def _sync(self, box, model, prompt_ids, params, headers, t0):
        st = self.state
        detok = IncrementalDetokenizer(box["target"].tokenizer, params.stop)
        text, n_out, finish, lps = [], 0, "stop", []
        gen = self._failover(box, model, prompt_ids, params, restartable=True)
        ttft = None
        try:
            async for it in gen:
                if it is RESTART:        # moved to another replica mid-generation
                    detok = IncrementalDetokenizer(box["target"].tokenizer, params.stop)
                    text, n_out, lps = [], 0, []
                    continue
                if it.token >= 0:
                    if ttft is None:
                        ttft = time.time() - t0
                    n_out += 1
                    text.append(detok.push(it.token))
                    if params.logprobs:
                        lps.append(logprob_item(box["target"].tokenizer, it.token, it.logprob,
                                                box.get("ids", False)))
                    if detok.stopped:
                        finish = "stop"
                        break
                if it.finish is not None:
                    finish = it.finish
                    break
        finally:
            await gen.aclose()
        text.append(detok.flush())
        target = box["target"]
        if finish.startswith("error"):
            self._record(target, model, "error", t0, len(prompt_ids), n_out, ttft,
                         headers.get(tracing.HEADER, ""))
            return write_error(502, "engine_failed", finish)
        self._record(target, model, "ok", t0, len(prompt_ids), n_out, ttft,
                         headers.get(tracing.HEADER, ""))
        choice = {"index": 0, "message": {"role": "assistant", "content": "".join(text)},
                  "finish_reason": finish if finish in ("stop", "length") else "stop"}
        if params.logprobs:
            choice["logprobs"] = {"content": lps}
        resp = {
            "id": "chatcmpl-" + uuid.uuid4().hex[:24], "object": "chat.completion",
            "created": int(time.time()), "model": model, "choices": [choice],
            "usage": {"prompt_tokens": len(prompt_ids), "completion_tokens": n_out,
                      "total_tokens": len(prompt_ids) + n_out}}
        r = write_json(200, resp)
        r.headers.update(headers)
        return r

    async def _stream(self, request, box, model, prompt_ids, params, include_usage, headers,
                      t0):
        st = self.state
        target = box["target"]
        resp = web.StreamResponse(status=200, headers={
            "Content-Type": "text/event-stream", "Cache-Control": "no-cache",
            "Connection": "keep-alive", **headers})
        await resp.prepare(request)
        chat_id = "chatcmpl-" + str(time.time_ns())
        created = int(time.time())
        head = ('data: {"id":"%s","object":"chat.completion.chunk","created":%d,"model":%s,'
                '"choices":[{"index":0,"delta":' % (chat_id, created, json.dumps(model)))
        detok = IncrementalDetokenizer(target.tokenizer, params.stop)
        n_out, finish, first = 0, "stop", True
        ttft = None
        gen = self._failover(box, model, prompt_ids, params)
        status = "ok"
        try:
            async for it in gen:
                if it.token >= 0:
                    n_out += 1
                    piece = detok.push(it.token)
                    # with logprobs every token gets its chunk (a partial UTF-8
                    # character streams as "" content next to its logprob)
                    if piece or first or params.logprobs:
                        if ttft is None:
                            ttft = time.time() - t0
                        role = '"role":"assistant",' if first else ""
                        first = False
                        lp = (',"logprobs":{"content":[%s]}' % dumps(logprob_item(
                            box["target"].tokenizer, it.token, it.logprob, box.get("ids", False)))
                            if params.logprobs else "")
                        await resp.write((head + '{%s"content":%s}%s}]}\n\n'
                                          % (role, json.dumps(piece, ensure_ascii=False), lp)
                                          ).encode())
                    if detok.stopped:
                        finish = "stop"
                        break
                if it.finish is not None:
                    finish = it.finish
                    break
            tail = detok.flush()
            if tail:
                await resp.write((head + '{"content":%s}}]}\n\n'
                                  % json.dumps(tail, ensure_ascii=False)).encode())
            if finish.startswith("error"):
                status = "error"
                finish = "error"
            final = {"id": chat_id, "object": "chat.completion.chunk", "created": created,
                     "model": model, "choices": [{"index": 0, "delta": {},
                                                  "finish_reason": finish}]}
            await resp.write(b"data: " + dumps(final).encode() + b"\n\n")
            if include_usage:
                usage = {"id": chat_id, "object": "chat.completion.chunk", "created": created,
                         "model": model, "choices": [],
                         "usage": {"prompt_tokens": len(prompt_ids), "completion_tokens": n_out,
                                   "total_tokens": len(prompt_ids) + n_out}}
                await resp.write(b"data: " + dumps(usage).encode() + b"\n\n")
            await resp.write(b"data: [DONE]\n\n")
        except (ConnectionResetError, ConnectionError):
            status = "client_gone"
        finally:
            await gen.aclose()
            self._record(box["target"], model, status, t0, len(prompt_ids), n_out, ttft,
                         headers.get(tracing.HEADER, ""))
        return resp

    def _record(self, target, model, status, t0, n_in, n_out, ttft, rid="", n=1):
        st = self.state
        elapsed = time.time() - t0
        # per-request span: TTFT = queue + prefill, decode = first -> last token
        tracing.record_span(
            "chat", rid, model=model, device_id=target.device_id, status=status, n=n,
            prompt_tokens=n_in, completion_tokens=n_out, total_ms=elapsed * 1e3,
            ttft_ms=None if ttft is None else ttft * 1e3,
            decode_ms=None if ttft is None else (elapsed - ttft) * 1e3,
            itl_ms=(elapsed - ttft) / (n_out - 1) * 1e3 if ttft is not None and n_out > 1
            else None)
        m = st.metrics
        m.chat_requests(model, target.device_id, status)
        if status in ("ok", "client_gone"):
            m.chat_duration(model, target.device_id, elapsed)
            m.chat_tokens(model, "local", n_in, n_out)
            if ttft is not None:
                m.ttft(model, ttft)
                if n_out > 1:
                    m.inter_token(model, (elapsed - ttft) / (n_out - 1))
        circuit = getattr(st, "circuit", None)
        if circuit is not None:
            circuit.record(target.device_id, status != "error")
        hook = getattr(st, "on_chat_done", None)
        if hook is not None:
            hook(model, n_in, n_out, int(elapsed * 1000), status)
