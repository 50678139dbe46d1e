"""Load generator for /v1/chat/completions (SSE) and /v1/embeddings.

Methodology follows the reference's probe harness
(scripts/probe_openrouter_models.py:113-123, 373-383): per request, TTFT =
request start -> first SSE chunk carrying content; completion tokens from the
stream's ``usage`` (stream_options.include_usage); p50/p95 by linear
interpolation.

Runs standalone (``python -m llm_mcp_amd.bench.loadgen --url ...``) or as the
client subprocess of bench.py: then it reads one command per line on stdin
("run" = one wave, "closed WARMUP_S DURATION_S" = a constant-concurrency
window, "open RATE WARMUP_S DURATION_S" = Poisson arrivals, "quit") and
answers one JSON line per command on stdout.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import random
import string
import sys
import time

import aiohttp


def percentile(xs: list[float], q: float) -> float:
    """Linear-interpolation percentile (same definition as the reference probe)."""
    if not xs:
        return 0.0
    s = sorted(xs)
    k = (len(s) - 1) * q / 100.0
    f = int(k)
    c = min(f + 1, len(s) - 1)
    return s[f] + (s[c] - s[f]) * (k - f)


_ALPHABET = string.ascii_letters + string.digits + "     "

# per-token inter-arrival gaps (SSE content chunk to the next one of the same
# stream) as a log-spaced histogram: 40 bins per decade from 10 us to 100 s,
# merged across load generators by summing; the per-request mean ITL hides a
# long prefill step that stalls every decoding stream once, this does not
GAP_BINS, GAP_LO, GAP_PER_DEC = 280, 1e-5, 40


def gap_bin(g: float) -> int:
    import math
    if g <= GAP_LO:
        return 0
    return min(GAP_BINS - 1, int(math.log10(g / GAP_LO) * GAP_PER_DEC))


def hist_percentile(h: list[int], q: float) -> float:
    """Upper edge (seconds) of the bin holding the q-th percentile of ``h``."""
    n = sum(h)
    if n == 0:
        return 0.0
    target, acc = n * q / 100.0, 0
    for i, c in enumerate(h):
        acc += c
        if acc >= target:
            return GAP_LO * 10 ** ((i + 1) / GAP_PER_DEC)
    return GAP_LO * 10 ** (GAP_BINS / GAP_PER_DEC)


def synthetic_prompt(n_chars: int, rng: random.Random) -> str:
    return "".join(rng.choices(_ALPHABET, k=n_chars))


_PROMPTS: dict = {}     # seed -> prompts of that wave, generated ahead during the previous wave


def wave_prompts(seed: int, concurrency: int, prompt_len: int) -> list[str]:
    got = _PROMPTS.pop((seed, concurrency, prompt_len), None)
    if got is not None:
        return got
    rng = random.Random(seed)
    return [synthetic_prompt(prompt_len, rng) for _ in range(concurrency)]


async def one_chat(session, url, model, prompt, max_tokens, temperature, top_p, ignore_eos=True,
                   gaps: list | None = None):
    body = {"model": model, "messages": [{"role": "user", "content": prompt}], "stream": True,
            "max_tokens": max_tokens, "temperature": temperature, "top_p": top_p,
            "ignore_eos": ignore_eos, "stream_options": {"include_usage": True}}
    t0 = time.perf_counter()
    ttft, last, toks, chunks = None, None, 0, 0
    async with session.post(url + "/v1/chat/completions", json=body) as r:
        if r.status != 200:
            raise RuntimeError(f"HTTP {r.status}: {await r.text()}")
        async for line in r.content:
            if not line.startswith(b"data: "):
                continue
            data = line[6:].strip()
            if data == b"[DONE]":
                break
            # JSON-decode only the chunks that can carry usage (a quote inside
            # generated text is escaped, so these keys only match as keys):
            # 256 streams x ~100 chunks/s each stay cheap for one client process
            if b'"usage"' in data:
                obj = json.loads(data)
                if obj.get("usage"):
                    toks = obj["usage"]["completion_tokens"]
                    continue
                ch = obj.get("choices") or []
                if not (ch and "content" in (ch[0].get("delta") or {})):
                    continue
            elif b'"content"' not in data:
                continue
            now = time.perf_counter()
            if ttft is None:
                ttft = now - t0
            elif gaps is not None:
                gaps[gap_bin(now - last)] += 1
            last = now
            chunks += 1
    t1 = time.perf_counter()
    return {"ttft": ttft or (t1 - t0), "latency": t1 - t0, "tokens": toks or chunks,
            "decode_s": (last - t0 - ttft) if (last and ttft) else 0.0}


async def wave(url, model, concurrency, prompt_len, max_tokens, temperature, top_p, seed,
               session=None):
    """One wave of ``concurrency`` concurrent streams.  ``session``: a
    ClientSession kept across waves (its keep-alive connections skip the
    reconnects at the start of the next wave), else a fresh one."""
    prompts = wave_prompts(seed, concurrency, prompt_len)
    # the next wave's prompts are generated while this one streams (the gap
    # between two timed waves then holds no client-side prompt generation)
    nxt = (seed + 1, concurrency, prompt_len)
    asyncio.get_running_loop().call_later(
        0.5, lambda: _PROMPTS.setdefault(nxt, wave_prompts(*nxt)))
    own = session is None
    s = session or new_session()
    gaps = [0] * GAP_BINS
    try:
        t0 = time.perf_counter()
        res = await asyncio.gather(*[one_chat(s, url, model, p, max_tokens, temperature, top_p,
                                              gaps=gaps)
                                     for p in prompts])
        el = time.perf_counter() - t0
    finally:
        if own:
            await s.close()
    ttfts = [r["ttft"] for r in res]
    tok = sum(r["tokens"] for r in res)
    itl = [r["decode_s"] / (r["tokens"] - 1) for r in res if r["tokens"] > 1]
    return {"elapsed": el, "tokens": tok, "requests": len(res), "ttfts": ttfts, "itls": itl,
            "gaps": gaps, "ttft_p50": percentile(ttfts, 50), "ttft_p95": percentile(ttfts, 95),
            "itl_p50": percentile(itl, 50), "tok_s": tok / el if el > 0 else 0.0}


async def closed_loop(url, model, concurrency, prompt_len, max_tokens, temperature, top_p, seed,
                      warmup_s: float, duration_s: float, session=None):
    """Constant concurrency: ``concurrency`` client loops, each sending its
    next request as soon as the previous stream ends, for ``warmup_s`` +
    ``duration_s`` seconds.  Throughput over the window counts every
    request's tokens in proportion to its overlap with the window (tokens
    spread over the stream's decode time); TTFT / ITL over the requests that
    START inside the window."""
    rng = random.Random(seed)
    t_start = time.perf_counter()
    w0, w1 = t_start + warmup_s, t_start + warmup_s + duration_s
    recs = []
    s = session or new_session()
    gaps = [0] * GAP_BINS

    async def client(k):
        while time.perf_counter() < w1:
            p = synthetic_prompt(prompt_len, rng)
            t0 = time.perf_counter()
            r = await one_chat(s, url, model, p, max_tokens, temperature, top_p,
                               gaps=gaps if t0 >= w0 else None)
            r["t0"] = t0
            recs.append(r)

    try:
        await asyncio.gather(*[client(k) for k in range(concurrency)])
    finally:
        if session is None:
            await s.close()
    return _window_summary(recs, w0, w1, duration_s, gaps)


async def open_loop(url, model, rate, prompt_len, max_tokens, temperature, top_p, seed,
                    warmup_s: float, duration_s: float, session=None):
    """Open loop: requests arrive as a Poisson process of ``rate`` per second
    (exponential gaps, seeded), each streamed to its end whatever else is in
    flight, for ``warmup_s`` + ``duration_s`` seconds; the window is summarised
    as in ``closed_loop``."""
    rng = random.Random(seed)
    t_start = time.perf_counter()
    w0, w1 = t_start + warmup_s, t_start + warmup_s + duration_s
    recs, tasks = [], []
    s = session or new_session()
    gaps = [0] * GAP_BINS

    async def one(p, t0):
        r = await one_chat(s, url, model, p, max_tokens, temperature, top_p,
                           gaps=gaps if t0 >= w0 else None)
        r["t0"] = t0
        recs.append(r)

    try:
        t_next = t_start
        while t_next < w1:
            now = time.perf_counter()
            if t_next > now:
                await asyncio.sleep(t_next - now)
            tasks.append(asyncio.ensure_future(one(synthetic_prompt(prompt_len, rng), t_next)))
            t_next += rng.expovariate(rate)
        await asyncio.gather(*tasks)
    finally:
        if session is None:
            await s.close()
    out = _window_summary(recs, w0, w1, duration_s, gaps)
    out["arrivals"] = len(tasks)
    return out


def _window_summary(recs, w0, w1, duration_s, gaps):
    tok = 0.0
    for r in recs:
        a, b = r["t0"] + r["ttft"], r["t0"] + r["latency"]     # token-producing span
        if b <= a:
            tok += r["tokens"] if w0 <= a < w1 else 0
            continue
        tok += r["tokens"] * max(0.0, min(b, w1) - max(a, w0)) / (b - a)
    inside = [r for r in recs if w0 <= r["t0"] < w1]
    ttfts = [r["ttft"] for r in inside]
    itl = [r["decode_s"] / (r["tokens"] - 1) for r in inside if r["tokens"] > 1]
    return {"elapsed": duration_s, "tokens": tok, "requests": len(inside), "ttfts": ttfts,
            "itls": itl, "gaps": gaps, "ttft_p50": percentile(ttfts, 50),
            "ttft_p95": percentile(ttfts, 95), "itl_p50": percentile(itl, 50),
            "itl_p95": percentile(itl, 95), "tok_s": tok / duration_s}


def new_session() -> aiohttp.ClientSession:
    return aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0),
                                 timeout=aiohttp.ClientTimeout(total=3600))


async def wait_ready(url, timeout=1800):
    t_end = time.time() + timeout
    async with aiohttp.ClientSession() as s:
        while time.time() < t_end:
            try:
                async with s.get(url + "/ready") as r:
                    if r.status == 200:
                        return True
            except Exception:
                pass
            await asyncio.sleep(0.5)
    return False


async def _make_session() -> aiohttp.ClientSession:
    return new_session()          # created inside the loop that will use it


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="http://127.0.0.1:8080")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--temperature", type=float, default=0.8)
    ap.add_argument("--top-p", type=float, default=0.95)
    ap.add_argument("--waves", type=int, default=1)
    ap.add_argument("--seed-base", type=int, default=0,
                    help="distinct per load-generator process (distinct prompts, no "
                         "accidental prefix-cache hits across generators)")
    ap.add_argument("--serve-stdin", action="store_true",
                    help="wait for 'run' commands on stdin (bench.py client mode)")
    a = ap.parse_args(argv)
    loop = asyncio.new_event_loop()
    if a.serve_stdin:
        ok = loop.run_until_complete(wait_ready(a.url))
        print(json.dumps({"ready": ok}), flush=True)
        session = loop.run_until_complete(_make_session())
        i = 0
        for line in sys.stdin:
            cmd = line.strip()
            if cmd == "quit":
                break
            if cmd.startswith("open"):
                _, rate, warm, dur = cmd.split()
                r = loop.run_until_complete(open_loop(
                    a.url, a.model, float(rate), a.prompt_len, a.max_tokens, a.temperature,
                    a.top_p, (a.seed_base << 20) + 777, float(warm), float(dur), session=session))
                print(json.dumps(r), flush=True)
                continue
            if cmd.startswith("closed"):
                _, warm, dur = cmd.split()
                r = loop.run_until_complete(closed_loop(
                    a.url, a.model, a.concurrency, a.prompt_len, a.max_tokens, a.temperature,
                    a.top_p, (a.seed_base << 20) + 999, float(warm), float(dur), session=session))
                print(json.dumps(r), flush=True)
                continue
            if cmd.startswith("run"):
                r = loop.run_until_complete(wave(a.url, a.model, a.concurrency, a.prompt_len,
                                                 a.max_tokens, a.temperature, a.top_p,
                                                 (a.seed_base << 20) + i, session=session))
                i += 1
                print(json.dumps(r), flush=True)
        loop.run_until_complete(session.close())
        return
    for i in range(a.waves):
        r = loop.run_until_complete(wave(a.url, a.model, a.concurrency, a.prompt_len,
                                         a.max_tokens, a.temperature, a.top_p,
                                         (a.seed_base << 20) + i))
        r.pop("ttfts")
        r.pop("itls")
        r.pop("gaps")
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
