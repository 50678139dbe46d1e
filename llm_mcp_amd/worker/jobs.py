"""Job-kind handlers of the GPU worker (reference: worker/llm_worker/main.py:330-519).

Every handler runs in-process on the worker's own engines -- no HTTP hop to
Ollama.  Kinds:
  engine.generate / ollama.generate   prompt or messages -> text (+ <think> split)
  engine.chat                         OpenAI-style messages -> text
  engine.embed / ollama.embed         prompt | input[] -> embedding(s)
  benchmark.{engine,ollama}.generate  synthetic decode benchmark -> tps, ttft,
                                      reported via ReportBenchmark
  benchmark.{engine,ollama}.embed     synthetic embedding benchmark
  openai.chat / openrouter.chat       cloud, only when LMX_ALLOW_CLOUD=1
  anything else                       echo {ok: true, echo: payload}
Result schema kept: {ok, response, thinking?, model, provider, device_id, tier,
tokens_in, tokens_out, cost: "X.XXXXX$", data}; metrics {ms, model, provider,
tokens_in, tokens_out} (consumed by RecordCost on completion).
"""
from __future__ import annotations

import asyncio
import os
import re
import time

from ..engine.engine import SamplingParams
from ..models.tokenizer import apply_chat_template

THINK_RE = re.compile(r"<think>(.*?)</think>", re.DOTALL)


class JobError(Exception):
    pass


def split_thinking(text: str) -> tuple[str, str]:
    m = THINK_RE.search(text)
    if not m:
        return "", text
    return m.group(1).strip(), (text[:m.start()] + text[m.end():]).strip()


def calc_cost(payload: dict, tokens_in: int, tokens_out: int) -> str:
    pin = float(payload.get("_price_in_1m") or 0)
    pout = float(payload.get("_price_out_1m") or 0)
    return f"{pin / 1e6 * tokens_in + pout / 1e6 * tokens_out:.5f}$"


def sampling_from_payload(payload: dict, default_max: int = 512,
                          ollama_defaults: bool = False) -> SamplingParams:
    """Job payload (+ Ollama ``options``) -> SamplingParams.  ``ollama.*``
    kinds get Ollama's generation defaults (repeat_penalty 1.1 over the last
    64 tokens), which the reference's jobs received from their Ollama
    backend (worker/llm_worker/main.py:222-243)."""
    o = dict(payload.get("options") or {})
    for k in ("temperature", "top_p", "top_k", "max_tokens", "stop", "seed", "presence_penalty",
              "frequency_penalty", "repetition_penalty"):
        if payload.get(k) is not None:
            o.setdefault(k, payload[k])
    stop = o.get("stop") or []
    if isinstance(stop, str):
        stop = [stop]
    max_tokens = o.get("max_tokens", o.get("num_predict", default_max))
    rep = o.get("repetition_penalty", o.get("repeat_penalty", 1.1 if ollama_defaults else 1.0))
    last_n = int(o.get("repeat_last_n", 64))
    return SamplingParams(temperature=float(o.get("temperature", 0.8)),
                          top_p=float(o.get("top_p", 1.0)), top_k=int(o.get("top_k", 0)),
                          max_tokens=max(1, int(max_tokens)), stop=list(stop),
                          seed=o.get("seed"), ignore_eos=bool(o.get("ignore_eos", False)),
                          repetition_penalty=float(rep),
                          presence_penalty=float(o.get("presence_penalty", 0.0)),
                          frequency_penalty=float(o.get("frequency_penalty", 0.0)),
                          penalty_last_n=64 if last_n < 0 else min(last_n, 64))


class JobRunner:
    """Executes claimed jobs against this worker's local models."""

    def __init__(self, registry, device_id: str, report_benchmark=None):
        self.registry = registry
        self.device_id = device_id
        self.report_benchmark = report_benchmark  # callable(**fields) or None

    def _model(self, name: str, kind: str):
        m = self.registry.select(name, kind) if name else None
        if m is None and not name:
            cands = [x for x in self.registry.all() if x.kind == kind]
            m = cands[0] if cands else None
        if m is None:
            raise JobError(f"model '{name}' ({kind}) is not served on {self.device_id}")
        return m

    async def _generate(self, m, prompt_ids, sp, progress: dict | None = None):
        """Run one request on the engine; ``progress`` (the agent's per-job
        report dict) is updated in place with tokens_out / ttft_ms."""
        from ..models.tokenizer import IncrementalDetokenizer
        detok = IncrementalDetokenizer(m.tokenizer, sp.stop)
        parts, n, ttft, t0 = [], 0, None, time.time()
        if progress is not None:
            progress.update(tokens_in=len(prompt_ids), tokens_out=0)
        fin = "stop"
        m.inflight += 1
        try:
            gen = m.engine.generate(prompt_ids, sp)
            try:
                async for it in gen:
                    if it.token >= 0:
                        if ttft is None:
                            ttft = time.time() - t0
                            if progress is not None:
                                progress["ttft_ms"] = int(ttft * 1000)
                        n += 1
                        if progress is not None:
                            progress["tokens_out"] = n
                        parts.append(detok.push(it.token))
                        if detok.stopped:
                            break
                    if it.finish is not None:
                        fin = it.finish
                        break
            finally:
                await gen.aclose()
        finally:
            m.inflight -= 1
        if fin.startswith("error"):
            raise JobError(fin)
        parts.append(detok.flush())
        el = time.time() - t0
        return "".join(parts), n, ttft or el, el, fin

    async def handle(self, kind: str, payload: dict,
                     progress: dict | None = None) -> tuple[dict, dict]:
        if kind in ("engine.generate", "ollama.generate", "engine.chat"):
            return await self.generate(payload, kind, progress)
        if kind in ("engine.embed", "ollama.embed"):
            return await self.embed(payload)
        if kind.startswith("benchmark.") and kind.endswith(".generate"):
            return await self.bench_generate(payload)
        if kind.startswith("benchmark.") and kind.endswith(".embed"):
            return await self.bench_embed(payload)
        if kind in ("openai.chat", "openrouter.chat"):
            from .cloud import cloud_chat
            return await cloud_chat(kind, payload)
        return {"ok": True, "echo": payload}, {"ms": 0}

    async def generate(self, payload: dict, kind: str, progress: dict | None = None):
        model = payload.get("model") or ""
        m = self._model(model, "chat")
        tok = m.tokenizer
        if payload.get("messages") and (kind == "engine.chat" or not payload.get("prompt")):
            ids = apply_chat_template(tok, payload["messages"])
        else:
            prompt = payload.get("prompt") or ""
            if not prompt:
                raise JobError("prompt_required")
            ids = tok.encode(prompt, add_bos=True)
        left = m.max_model_len - len(ids) - 1
        if left < 1:
            raise JobError("context_length_exceeded")
        sp = sampling_from_payload(payload, ollama_defaults=kind.startswith("ollama."))
        sp.max_tokens = min(sp.max_tokens, left)
        text, n_out, ttft, el, fin = await self._generate(m, ids, sp, progress)
        thinking = ""
        if "<think>" in text:
            thinking, text = split_thinking(text)
        n_in = len(ids)
        res = {"ok": True, "response": text, "model": m.model_id, "provider": "local",
               "device_id": m.device_id, "tier": payload.get("_tier", ""),
               "tokens_in": n_in, "tokens_out": n_out, "cost": calc_cost(payload, n_in, n_out),
               "data": {"done_reason": fin, "prompt_eval_count": n_in, "eval_count": n_out,
                        "ttft_ms": int(ttft * 1000), "total_ms": int(el * 1000),
                        "tps": round(n_out / max(1e-6, el - ttft), 2) if n_out > 1 else None}}
        if thinking and payload.get("thinking", True):
            res["thinking"] = thinking
        return res, {"ms": int(el * 1000), "model": m.model_id, "provider": "local",
                     "tokens_in": n_in, "tokens_out": n_out}

    async def embed(self, payload: dict):
        m = self._model(payload.get("model") or "", "embed")
        inp = payload.get("input", payload.get("prompt"))
        texts = [inp] if isinstance(inp, str) else [t for t in (inp or []) if isinstance(t, str)]
        if not texts:
            raise JobError("prompt_required")
        seqs = [m.tokenizer.encode(t, add_bos=True) + list(m.tokenizer.eos_ids[:1])
                for t in texts]
        t0 = time.time()
        vecs = await m.engine.embed(seqs, payload.get("dimensions"))
        vecs = [list(map(float, v)) for v in vecs]      # JSON job result
        ms = int((time.time() - t0) * 1000)
        data = {"embedding": vecs[0]} if isinstance(inp, str) else {"embeddings": vecs}
        return ({"ok": True, "provider": "local", "model": m.model_id, "device_id": m.device_id,
                 "data": data},
                {"ms": ms, "model": m.model_id, "provider": "local",
                 "tokens_in": sum(len(s) for s in seqs), "tokens_out": 0})

    async def bench_generate(self, payload: dict):
        m = self._model(payload.get("model") or "", "chat")
        n_prompt = int(payload.get("prompt_tokens", 128))
        max_tokens = int(payload.get("max_tokens", 128))
        conc = max(1, int(payload.get("concurrency", 1)))
        if payload.get("prompt"):
            ids = m.tokenizer.encode(payload["prompt"], add_bos=True)
        else:
            ids = [(i * 7919) % 250 + 3 for i in range(n_prompt)]
        sp = SamplingParams(temperature=0.0, max_tokens=max_tokens, ignore_eos=True)
        t0 = time.time()
        outs = await asyncio.gather(*[self._generate(m, ids, sp) for _ in range(conc)])
        el = time.time() - t0
        n_out = sum(o[1] for o in outs)
        ttft = min(o[2] for o in outs)
        decode = max(1e-6, max(o[3] - o[2] for o in outs))
        tps = round(n_out / decode, 2)
        lat = int(el * 1000)
        if self.report_benchmark is not None:
            await asyncio.to_thread(self.report_benchmark, device_id=m.device_id,
                                    model_id=m.model_id, task_type="generate",
                                    tokens_in=len(ids) * conc, tokens_out=n_out, latency_ms=lat,
                                    tps=tps, meta={"ttft_ms": int(ttft * 1000),
                                                   "concurrency": conc})
        return ({"ok": True, "provider": "local", "model": m.model_id, "device_id": m.device_id,
                 "tokens_in": len(ids) * conc, "tokens_out": n_out, "latency_ms": lat,
                 "ttft_ms": int(ttft * 1000), "tps": tps},
                {"ms": lat, "model": m.model_id, "provider": "local"})

    async def bench_embed(self, payload: dict):
        m = self._model(payload.get("model") or "", "embed")
        n = int(payload.get("prompt_tokens", 128))
        conc = max(1, int(payload.get("concurrency", 16)))
        seqs = [[(i * 31 + j) % 250 + 3 for i in range(n)] for j in range(conc)]
        t0 = time.time()
        await m.engine.embed(seqs, None)
        el = time.time() - t0
        lat = int(el * 1000)
        tps = round(n * conc / max(el, 1e-6), 1)
        if self.report_benchmark is not None:
            await asyncio.to_thread(self.report_benchmark, device_id=m.device_id,
                                    model_id=m.model_id, task_type="embed",
                                    tokens_in=n * conc, tokens_out=0, latency_ms=lat, tps=tps,
                                    meta={"sequences": conc})
        return ({"ok": True, "provider": "local", "model": m.model_id, "tokens_in": n * conc,
                 "tokens_out": 0, "latency_ms": lat, "tps": tps},
                {"ms": lat, "model": m.model_id, "provider": "local"})


ENGINE_KINDS = ["engine.generate", "engine.chat", "engine.embed", "ollama.generate",
                "ollama.embed", "benchmark.engine.generate", "benchmark.engine.embed",
                "benchmark.ollama.generate", "benchmark.ollama.embed"]


def default_kinds() -> list[str]:
    env = os.environ.get("WORKER_KINDS", "").strip()
    if env:
        return [k.strip() for k in env.split(",") if k.strip()]
    kinds = list(ENGINE_KINDS)
    if os.environ.get("LMX_ALLOW_CLOUD", "0") == "1":
        kinds += ["openai.chat", "openrouter.chat"]
    return kinds
