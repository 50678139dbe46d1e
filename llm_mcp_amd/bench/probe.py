"""Async-job probe harness: synthetic requests through the job queue.

Behavioural counterpart of the reference's
scripts/probe_openrouter_models.py:153-220,244-400 (C19): for every model x
run it submits ``POST /v1/llm/request``, polls ``GET /v1/jobs/{id}`` until
the job settles, and derives latency, tokens (``tokens_in/out`` from the
result, else chars/4 as the reference does) and tokens/s.  Differences:

* the default target is the local GPU engines (the reference only probes
  OpenRouter); ``--cloud`` probes the curated cloud catalogue instead and
  sends ``force_cloud`` (needs LMX_ALLOW_CLOUD=1 on the core);
* each successful run is recorded as a ``benchmarks`` row through the gRPC
  ``ReportBenchmark`` call (``--grpc``) rather than a direct SQL INSERT, so
  it works against either store backend; the device is the one the job ran
  on (result ``device_id``) or ``cloud-openrouter``;
* the summary (p50/p95 latency and tps per model, linear-interpolation
  percentiles as the reference) is written as JSON to ``--out``.

    python -m llm_mcp_amd.bench.probe --base-url http://127.0.0.1:8080 \\
        --models llama-3-8b,nomic-embed-text --runs-per-model 3 --grpc 127.0.0.1:9090
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import time
from dataclasses import asdict, dataclass, field

import aiohttp

from .loadgen import percentile

PROBE_PROMPT = ("Summarise in two sentences why paged KV caches help continuous batching "
                "on GPUs with large HBM capacity.")


@dataclass
class ProbeRun:
    model: str
    run: int
    job_id: str = ""
    status: str = ""
    ok: bool = False
    latency_ms: float = 0.0
    tokens_in: int = 0
    tokens_out: int = 0
    tps: float = 0.0
    device_id: str = ""
    provider: str = ""
    error: str = ""
    meta: dict = field(default_factory=dict)


def output_text(result: dict) -> str:
    """The generated text of a job result, whatever the job kind put it under."""
    for k in ("response", "text", "output", "content"):
        v = result.get(k)
        if isinstance(v, str) and v:
            return v
    data = result.get("data")
    if isinstance(data, dict):
        for k in ("response", "text"):
            if isinstance(data.get(k), str):
                return data[k]
        ch = data.get("choices")
        if isinstance(ch, list) and ch:
            msg = ch[0].get("message") or {}
            if isinstance(msg.get("content"), str):
                return msg["content"]
    return ""


def usage(result: dict, prompt: str) -> tuple[int, int]:
    """(tokens_in, tokens_out): the result's counts, else chars/4."""
    ti, to = int(result.get("tokens_in") or 0), int(result.get("tokens_out") or 0)
    if ti <= 0:
        ti = max(1, len(prompt) // 4)
    if to <= 0:
        to = max(0, len(output_text(result)) // 4)
    return ti, to


async def _wait_job(s: aiohttp.ClientSession, base: str, jid: str, timeout: float,
                    poll: float) -> dict:
    end = time.monotonic() + timeout
    while True:
        async with s.get(f"{base}/v1/jobs/{jid}") as r:
            job = await r.json()
        if job.get("status") in ("done", "error"):
            return job
        if time.monotonic() > end:
            job["status"] = "timeout"
            return job
        await asyncio.sleep(poll)


async def probe_one(s: aiohttp.ClientSession, base: str, model: str, run: int, a) -> ProbeRun:
    pr = ProbeRun(model=model, run=run)
    body = {"model": model, "prompt": a.prompt, "max_tokens": a.max_tokens,
            "source": "probe"}
    if a.cloud:
        body["force_cloud"] = True
    if a.task:
        body["task"] = a.task
    if a.quality:
        body["quality"] = a.quality
    t0 = time.perf_counter()
    try:
        async with s.post(f"{base}/v1/llm/request", json=body) as r:
            sub = await r.json()
            if r.status != 202:
                pr.status, pr.error = "rejected", sub.get("message") or sub.get("error", "")
                return pr
        pr.job_id, pr.provider = sub["job_id"], sub.get("provider", "")
        job = await _wait_job(s, base, pr.job_id, a.job_timeout_sec, a.poll_sec)
    except (aiohttp.ClientError, asyncio.TimeoutError, KeyError) as ex:
        pr.status, pr.error = "http_error", str(ex)
        return pr
    pr.latency_ms = (time.perf_counter() - t0) * 1e3
    pr.status = job.get("status", "")
    res = job.get("result") or {}
    if isinstance(res, str):
        try:
            res = json.loads(res)
        except ValueError:
            res = {"response": res}
    pr.ok = pr.status == "done" and res.get("ok", True) is not False
    pr.error = str(job.get("error") or "")
    pr.tokens_in, pr.tokens_out = usage(res, a.prompt)
    pr.tps = pr.tokens_out / (pr.latency_ms / 1e3) if pr.latency_ms > 0 else 0.0
    pr.device_id = str(res.get("device_id") or ("cloud-openrouter" if a.cloud else ""))
    pr.meta = {"attempts": job.get("attempts"), "kind": job.get("kind")}
    return pr


def summarise(runs: list[ProbeRun]) -> dict:
    out: dict[str, dict] = {}
    for m in dict.fromkeys(r.model for r in runs):
        rs = [r for r in runs if r.model == m]
        ok = [r for r in rs if r.ok]
        lat, tps = [r.latency_ms for r in ok], [r.tps for r in ok]
        out[m] = {"runs": len(rs), "ok": len(ok),
                  "latency_p50_ms": round(percentile(lat, 50), 1),
                  "latency_p95_ms": round(percentile(lat, 95), 1),
                  "tps_p50": round(percentile(tps, 50), 2),
                  "tps_p95": round(percentile(tps, 95), 2),
                  "errors": sorted({r.error or r.status for r in rs if not r.ok})}
    return out


def record(runs: list[ProbeRun], report) -> int:
    """Write one benchmarks row per successful run via ``report`` (the gRPC
    client's ``report_benchmark`` signature)."""
    n = 0
    for r in runs:
        if not r.ok:
            continue
        report(r.device_id or "unknown", r.model, "probe.generate", r.tokens_in, r.tokens_out,
               int(r.latency_ms), float(r.tps), {"job_id": r.job_id, "provider": r.provider,
                                                 "source": "probe"})
        n += 1
    return n


def load_models(a) -> list[str]:
    if a.models:
        return [m.strip() for m in a.models.split(",") if m.strip()]
    if a.cloud:
        from ..planner.catalog import load_curated
        path = a.config or os.path.join(os.path.dirname(__file__), "..", "config",
                                        "curated_cloud_models.yaml")
        return load_curated(path)
    return ["llama-3-8b"]


async def run_probe(a) -> tuple[list[ProbeRun], dict]:
    base = a.base_url.rstrip("/")
    models = load_models(a)
    tmo = aiohttp.ClientTimeout(total=a.http_timeout_sec)
    runs: list[ProbeRun] = []
    async with aiohttp.ClientSession(timeout=tmo) as s:
        for m in models:
            for i in range(a.runs_per_model):
                pr = await probe_one(s, base, m, i, a)
                runs.append(pr)
                print(json.dumps({"probe": m, "run": i, "status": pr.status,
                                  "latency_ms": round(pr.latency_ms, 1),
                                  "tps": round(pr.tps, 2)}), flush=True)
    return runs, summarise(runs)


def parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--base-url", default=os.getenv("LLM_CORE_URL", "http://127.0.0.1:8080"))
    ap.add_argument("--models", default="", help="comma list (default: llama-3-8b, or the "
                    "curated catalogue with --cloud)")
    ap.add_argument("--cloud", action="store_true", help="probe curated cloud models")
    ap.add_argument("--config", default=None, help="curated catalogue YAML (--cloud)")
    ap.add_argument("--task", default="", help="router task hint (chat, reason, embed, ...)")
    ap.add_argument("--quality", default="", help="router quality tier (turbo ... max)")
    ap.add_argument("--prompt", default=PROBE_PROMPT)
    ap.add_argument("--runs-per-model", type=int, default=3)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--poll-sec", type=float, default=1.2)
    ap.add_argument("--job-timeout-sec", type=float, default=180.0)
    ap.add_argument("--http-timeout-sec", type=float, default=20.0)
    ap.add_argument("--grpc", default="", help="core gRPC address: record benchmarks rows")
    ap.add_argument("--out", default="artifacts/probe", help="directory for the JSON report")
    ap.add_argument("--dry-run", action="store_true")
    return ap


def main(argv=None) -> int:
    a = parser().parse_args(argv)
    if a.dry_run:
        print(json.dumps({"models": load_models(a), "runs_per_model": a.runs_per_model,
                          "base_url": a.base_url}))
        return 0
    runs, summary = asyncio.run(run_probe(a))
    recorded = 0
    if a.grpc:
        from ..rpc.client import CoreClient
        c = CoreClient(a.grpc)
        try:
            recorded = record(runs, c.report_benchmark)
        finally:
            c.close()
    os.makedirs(a.out, exist_ok=True)
    path = os.path.join(a.out, f"probe_{time.strftime('%Y%m%dT%H%M%S')}.json")
    with open(path, "w") as f:
        json.dump({"summary": summary, "runs": [asdict(r) for r in runs],
                   "recorded": recorded}, f, indent=1)
    print(json.dumps({"summary": summary, "recorded": recorded, "report": path}))
    return 0 if all(v["ok"] for v in summary.values()) else 1


if __name__ == "__main__":
    raise SystemExit(main())
