"""Benchmarks for the BASELINE.json configs other than the headline chat SSE
run (bench.py):

  queue   submit -> claim -> heartbeat -> complete with echo workers on CPU
          (config 1: plumbing, no GPU).  Core gRPC server + W worker agents
          in one process; reports jobs/s and claim / end-to-end latency.
          ``--store postgres`` uses DB_DSN (none in this image).
  embed   /v1/embeddings nomic-embed-text bf16 on one GPU (config 2): API
          process + GPU worker process (sync path over the engine socket) +
          this process as the client; embeddings/s and p50/p95 latency.
  mixed   mixed chat + embeddings jobs at 256 concurrent jobs through the
          lease scheduler (config 5, on the GPUs given with --gpus): the
          production launcher ``python -m llm_mcp_amd serve`` + async jobs
          submitted over HTTP and awaited on the job SSE stream; jobs/s,
          p50/p95 latency, error rate.

Methodology follows the reference's probe harness (p50/p95 by linear
interpolation, scripts/probe_openrouter_models.py:113-123).  This process
never initialises the GPU: every GPU user is a child process.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import socket
import signal
import subprocess
import sys
import threading
import time

from .loadgen import percentile, synthetic_prompt


def _log(msg: str) -> None:
    print(f"[serving_bench] {msg}", file=sys.stderr, flush=True)


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _wait_http(url: str, path: str = "/health", timeout: float = 900) -> None:
    import aiohttp
    t_end = time.time() + timeout
    async with aiohttp.ClientSession() as s:
        while time.time() < t_end:
            try:
                async with s.get(url + path) as r:
                    if r.status == 200:
                        return
            except Exception:
                pass
            await asyncio.sleep(0.5)
            if int(time.time()) % 15 == 0:
                _log(f"waiting for {url}{path}")
    raise TimeoutError(f"{url}{path} never became ready")


# ------------------------------------------------------------------ queue ----
def bench_queue(a) -> dict:
    from ..api.core import CoreState, open_store
    from ..api.registry import ModelRegistry
    from ..rpc.client import CoreClient
    from ..rpc.server import start_grpc
    from ..worker.agent import WorkerAgent
    from ..worker.jobs import JobRunner

    st = CoreState(store=open_store(a.store))
    loop = asyncio.new_event_loop()
    box = {}

    def serve():
        asyncio.set_event_loop(loop)
        box["srv"], box["port"] = loop.run_until_complete(start_grpc(st, "127.0.0.1:0"))
        loop.run_forever()

    threading.Thread(target=serve, daemon=True).start()
    while "port" not in box:
        time.sleep(0.01)
    addr = f"127.0.0.1:{box['port']}"
    client = CoreClient(addr)
    # claim-latency probe on a populated queue (reference: ~19 ms with Postgres)
    n_probe = 200
    for i in range(n_probe + a.jobs):
        client.submit("echo", {"i": i}, source="probe")
    lat = []
    for _ in range(n_probe):
        t0 = time.perf_counter()
        j = client.claim("probe", lease_seconds=30)
        lat.append(time.perf_counter() - t0)
        if j:
            client.complete("probe", j["id"], {"ok": True}, attempt_id=j.get("attempt_id", ""))
    # throughput: W agents drain a.jobs queued behind the rest end to end
    ids = [client.submit("echo", {"i": i}, source="bench") for i in range(a.jobs)]
    a.jobs *= 2

    async def drain():
        agents = [WorkerAgent(CoreClient(addr), JobRunner(ModelRegistry(), f"cpu{w}"),
                              f"cpu{w}", worker_id=f"w{w}", lease_s=30, capacity=a.capacity)
                  for w in range(a.workers)]
        per = a.jobs // a.workers
        await asyncio.gather(*[ag.run(max_jobs=per + (1 if w < a.jobs % a.workers else 0))
                               for w, ag in enumerate(agents)])

    t0 = time.perf_counter()
    asyncio.new_event_loop().run_until_complete(drain())
    el = time.perf_counter() - t0
    done = sum(1 for i in ids if client.get(i)["status"] == "done")
    loop.call_soon_threadsafe(loop.stop)
    return {"config": "queue plumbing: submit->claim->heartbeat->complete, echo workers, CPU",
            "store": st.store.backend, "jobs": a.jobs, "workers": a.workers, "done": done,
            "jobs_per_s": round(a.jobs / el, 1),
            "claim_p50_ms": round(percentile(lat, 50) * 1e3, 3),
            "claim_p95_ms": round(percentile(lat, 95) * 1e3, 3)}


# ------------------------------------------------------------------ embed ----
async def _embed_load(url, model, concurrency, requests, batch, chars, seed=0):
    import aiohttp
    rng = random.Random(seed)
    docs = [synthetic_prompt(chars, rng) for _ in range(64)]
    lat = []
    sem = asyncio.Semaphore(concurrency)

    async def one(s, i):
        inp = [docs[(i * batch + k) % len(docs)] for k in range(batch)]
        async with sem:
            t0 = time.perf_counter()
            async with s.post(url + "/v1/embeddings", json={"model": model, "input": inp}) as r:
                body = await r.json()
                if r.status != 200:
                    raise RuntimeError(f"HTTP {r.status}: {body}")
            lat.append(time.perf_counter() - t0)
            return len(body["data"]), body["usage"]["prompt_tokens"]

    async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0)) as s:
        await asyncio.gather(*[one(s, i) for i in range(min(8, requests))])   # warm-up
        lat.clear()
        t0 = time.perf_counter()
        res = await asyncio.gather(*[one(s, i) for i in range(requests)])
        el = time.perf_counter() - t0
    n = sum(r[0] for r in res)
    toks = sum(r[1] for r in res)
    return {"embeddings": n, "tokens": toks, "elapsed_s": round(el, 3),
            "embeddings_per_s": round(n / el, 1), "tokens_per_s": round(toks / el, 1),
            "p50_ms": round(percentile(lat, 50) * 1e3, 2),
            "p95_ms": round(percentile(lat, 95) * 1e3, 2)}


def bench_embed(a) -> dict:
    sock = f"/tmp/lmx-embbench-{os.getpid()}.sock"
    port = _port()
    env = dict(os.environ)
    worker = subprocess.Popen([sys.executable, "-m", "llm_mcp_amd.worker.main", "--gpu",
                               str(a.gpu), "--chat-model", "", "--embed-model", a.model,
                               "--socket", sock, "--no-jobs"], env=env)
    api = subprocess.Popen([sys.executable, "-m", "llm_mcp_amd.api.serve", "--port", str(port),
                            "--engine", f"{a.model}=unix:{sock},device=gpu{a.gpu}"],
                           env=env, stdout=subprocess.DEVNULL)
    url = f"http://127.0.0.1:{port}"
    try:
        loop = asyncio.new_event_loop()
        loop.run_until_complete(_wait_http(url, "/ready"))
        out = {"config": "/v1/embeddings nomic-embed-text bf16, 1x MI355X (sync path)",
               "model": a.model, "concurrency": a.concurrency, "batch": a.batch,
               "doc_chars": a.chars}
        out.update(loop.run_until_complete(
            _embed_load(url, a.model, a.concurrency, a.requests, a.batch, a.chars)))
        out["single_p50"] = loop.run_until_complete(
            _embed_load(url, a.model, 1, 64, 1, a.chars))["p50_ms"]
        return out
    finally:
        for p in (api, worker):
            p.terminate()
        for p in (api, worker):
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()


# ------------------------------------------------------------------ mixed ----
async def _mixed_load(url, chat_model, embed_model, jobs, concurrency, embed_every, max_tokens,
                      prompt_chars, sync_every=0):
    """``sync_every`` k > 0: every k-th request is a synchronous
    /v1/chat/completions call (replica selection + circuit breaker on the
    hot path) instead of an async job."""
    import aiohttp
    rng = random.Random(1)
    sem = asyncio.Semaphore(concurrency)
    lat, errs, kinds = [], [], {}
    per_dev: dict[str, int] = {}
    done_at: list[tuple[float, str]] = []     # (monotonic time, device) per finished job
    requeued = [0]
    sync = {"ok": 0, "error": 0}

    async def one_sync(s, i):
        body = {"model": chat_model, "max_tokens": max_tokens, "temperature": 0.8,
                "ignore_eos": True,
                "messages": [{"role": "user", "content": synthetic_prompt(prompt_chars, rng)}]}
        async with sem:
            t0 = time.perf_counter()
            try:
                async with s.post(url + "/v1/chat/completions", json=body) as r:
                    ok = r.status == 200
                    await r.read()
            except aiohttp.ClientError:
                ok = False
            lat.append(time.perf_counter() - t0)
            sync["ok" if ok else "error"] += 1
            kinds["chat.sync"] = kinds.get("chat.sync", 0) + 1

    async def one(s, i):
        if sync_every and i % sync_every == 1:
            return await one_sync(s, i)
        if i % embed_every == 0:
            kind, payload = "engine.embed", {"model": embed_model,
                                             "prompt": synthetic_prompt(prompt_chars, rng)}
        else:
            kind, payload = "engine.generate", {
                "model": chat_model, "prompt": synthetic_prompt(prompt_chars, rng),
                "options": {"max_tokens": max_tokens, "temperature": 0.8, "ignore_eos": True}}
        async with sem:
            t0 = time.perf_counter()
            async with s.post(url + "/v1/jobs", json={"kind": kind, "payload": payload,
                                                      "source": "bench"}) as r:
                jid = (await r.json())["job_id"]
            status = None
            async with s.get(url + f"/v1/jobs/{jid}/stream") as r:
                async for line in r.content:
                    if line.startswith(b"data: "):
                        d = json.loads(line[6:])
                        status = d.get("status", status)
                        if status in ("done", "error"):
                            break
            lat.append(time.perf_counter() - t0)
            kinds[kind] = kinds.get(kind, 0) + 1
            if status != "done":
                errs.append(jid)
            else:
                async with s.get(url + f"/v1/jobs/{jid}") as r:
                    jj = await r.json()
                d = ((jj.get("result") or {}).get("device_id") or jj.get("device_id") or "?")
                per_dev[d] = per_dev.get(d, 0) + 1
                done_at.append((time.monotonic(), d))
                requeued[0] += int((jj.get("attempts") or 1) > 1)
            if len(lat) % 64 == 0:
                _log(f"{len(lat)}/{jobs} jobs finished, {len(errs)} errors")

    async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0),
                                     timeout=aiohttp.ClientTimeout(total=3600)) as s:
        t0 = time.perf_counter()
        t0_mono = time.monotonic()
        await asyncio.gather(*[one(s, i) for i in range(jobs)])
        el = time.perf_counter() - t0
    n_async = jobs - sync["ok"] - sync["error"]
    return {"jobs": jobs, "by_kind": kinds, "elapsed_s": round(el, 2),
            "jobs_per_s": round(jobs / el, 2), "p50_s": round(percentile(lat, 50), 3),
            "p95_s": round(percentile(lat, 95), 3),
            "error_rate": round(len(errs) / max(1, n_async), 4),
            "jobs_done_by_device": per_dev, "jobs_requeued": requeued[0],
            "sync_chat": sync, "_done_at": done_at, "_t0": t0_mono}


def bench_mixed(a) -> dict:
    port, gport = _port(), _port()
    env = dict(os.environ, LMX_STORE=a.store)
    if a.fault:
        env.update(LMX_FAULT=a.fault, LMX_FAULT_DEVICE=a.fault_device,
                   LMX_FAULT_LIVES=str(a.fault_lives))
    cmd = [sys.executable, "-m", "llm_mcp_amd", "serve", "--gpus", a.gpus, "--http",
           f"127.0.0.1:{port}", "--grpc", f"127.0.0.1:{gport}", "--chat-model", a.chat_model,
           "--embed-model", a.model, "--max-num-seqs", str(a.concurrency),
           "--replicas-per-gpu", str(a.replicas_per_gpu)]
    if a.replicas_per_gpu > 1:
        cmd += ["--kv-fraction", str(round(0.5 / a.replicas_per_gpu, 3))]
    if a.cpu:
        cmd += ["--cpu"]
    core = subprocess.Popen(cmd, env=env, start_new_session=True)
    url = f"http://127.0.0.1:{port}"
    try:
        loop = asyncio.new_event_loop()
        loop.run_until_complete(_wait_http(url, "/health"))
        # workers register once their engines are up
        n_workers = len(a.gpus.split(",")) * max(1, a.replicas_per_gpu)
        loop.run_until_complete(_wait_workers(url, n_workers))
        loop.run_until_complete(_wait_http(url, "/ready"))
        out = {"config": "mixed chat + embeddings jobs through the lease scheduler",
               "gpus": a.gpus, "replicas_per_gpu": a.replicas_per_gpu,
               "concurrency": a.concurrency, "chat_model": a.chat_model,
               "embed_model": a.model, "embed_share": round(1 / a.embed_every, 3),
               "sync_every": a.sync_every, "max_tokens": a.max_tokens,
               "fault": a.fault, "fault_device": a.fault_device}
        circ: dict[str, set] = {}
        trips: dict[str, int] = {}
        status_seen: dict[str, set] = {}

        async def poll_dashboard(s):
            async with s.get(url + "/v1/dashboard") as r:
                d = await r.json()
            for dev in d.get("devices") or []:
                k = dev.get("id", "?")
                circ.setdefault(k, set()).add(dev.get("circuit", "ok"))
                status_seen.setdefault(k, set()).add(dev.get("status", "?"))
                trips[k] = max(trips.get(k, 0), int(dev.get("circuit_trips") or 0))

        # fault-recovery timeline (monotonic seconds): every change of a
        # device's circuit / status and of a worker's alive flag / restarts
        timeline: list[tuple[float, str, str, str]] = []
        last: dict[tuple[str, str], str] = {}

        def note(key, what, val):
            if last.get((key, what)) != val:
                last[(key, what)] = val
                timeline.append((time.monotonic(), key, what, val))

        async def watch_circuit():
            import aiohttp
            async with aiohttp.ClientSession() as s:
                while True:
                    try:
                        async with s.get(url + "/v1/dashboard") as r:
                            d = await r.json()
                        for dev in d.get("devices") or []:
                            k = dev.get("id", "?")
                            circ.setdefault(k, set()).add(dev.get("circuit", "ok"))
                            status_seen.setdefault(k, set()).add(dev.get("status", "?"))
                            trips[k] = max(trips.get(k, 0), int(dev.get("circuit_trips") or 0))
                            note(k, "circuit", str(dev.get("circuit", "ok")))
                            note(k, "status", str(dev.get("status", "?")))
                        async with s.get(url + "/v1/debug/workers") as r:
                            for w in (await r.json()).get("workers") or []:
                                note(w.get("name", "?"), "alive", str(bool(w.get("alive"))))
                                note(w.get("name", "?"), "restarts", str(w.get("restarts", 0)))
                    except Exception:
                        pass
                    # fine-grained only when a fault's recovery is being timed
                    await asyncio.sleep(0.1 if a.fault else 0.5)

        async def run():
            w = asyncio.ensure_future(watch_circuit())
            try:
                return await _mixed_load(url, a.chat_model, a.model, a.jobs, a.concurrency,
                                         a.embed_every, a.max_tokens, a.chars, a.sync_every)
            finally:
                w.cancel()
        res = loop.run_until_complete(run())
        done_at, t0m = res.pop("_done_at"), res.pop("_t0")
        out.update(res)
        if a.fault:
            out["recovery"] = _recovery(timeline, done_at, t0m, a.fault_device)

        async def final_poll():
            import aiohttp
            async with aiohttp.ClientSession() as s:
                await poll_dashboard(s)
        loop.run_until_complete(final_poll())
        out["circuit_states_seen"] = {k: sorted(v) for k, v in circ.items()}
        # breaker trips (ok -> degraded transitions) counted by the core itself
        out["circuit_trips"] = trips
        out["device_status_seen"] = {k: sorted(v) for k, v in status_seen.items()}

        async def workers():
            import aiohttp
            async with aiohttp.ClientSession() as s:
                async with s.get(url + "/v1/debug/workers") as r:
                    return (await r.json()).get("workers")
        out["workers"] = loop.run_until_complete(workers())
        if a.await_recovery > 0:
            # after the load: how long until every supervised worker is alive
            # again and its device back online (the restarted worker
            # re-registered) -- reported, never part of the timed window
            t_rec = time.perf_counter()
            rec = None
            run_status = {k: sorted(v) for k, v in status_seen.items()}
            while time.perf_counter() - t_rec < a.await_recovery:
                ws = loop.run_until_complete(workers()) or []
                status_seen.clear()                 # current statuses only
                loop.run_until_complete(final_poll())
                online = all(v == {"online"} for v in status_seen.values())
                if ws and all(w.get("alive") for w in ws) and online:
                    rec = round(time.perf_counter() - t_rec, 1)
                    break
                time.sleep(1.0)
            out["device_status_seen"] = run_status
            out["recovered_after_s"] = rec
            out["workers_after_recovery"] = loop.run_until_complete(workers())
            out["device_status_after_recovery"] = {k: sorted(v) for k, v in status_seen.items()}
        return out
    finally:
        _stop_group(core)


def _stop_group(core: subprocess.Popen, grace_s: float = 60.0) -> None:
    """Stop the core and its worker processes.  The core stops its workers
    itself (SIGTERM, then a wait); if it has not exited after ``grace_s`` the
    whole process group it leads (``start_new_session``) gets SIGTERM -- each
    worker then still exits through its own handler, so a profiler attached
    to it writes its trace -- and SIGKILL only after a second grace."""
    core.terminate()
    try:
        core.wait(timeout=grace_s)
        return
    except subprocess.TimeoutExpired:
        pass
    for sig, wait in ((signal.SIGTERM, 30.0), (signal.SIGKILL, 10.0)):
        try:
            os.killpg(core.pid, sig)
        except ProcessLookupError:
            return
        try:
            core.wait(timeout=wait)
            return
        except subprocess.TimeoutExpired:
            pass


def _recovery(timeline, done_at, t0, fault_device: str) -> dict:
    """Fault -> recovery phases of the faulty device (seconds from the load's
    start): its last job served before the fault, the breaker trip, the
    worker's death and restart, the device back online, and its first job
    served after the restart.  ``recovery_s`` = fault (last good job) ->
    first job served by the replacement."""
    def first(pred, after=0.0):
        return next((round(t - t0, 2) for t, k, w, v in timeline
                     if t - t0 >= after and pred(k, w, v)), None)

    dev = fault_device
    died = first(lambda k, w, v: w == "alive" and v == "False")
    restarted = first(lambda k, w, v: w == "restarts" and v not in ("0", "None"))
    trip = first(lambda k, w, v: k.endswith(dev) and w == "circuit" and v == "degraded")
    mine = sorted(t - t0 for t, d in done_at if d.endswith(dev))
    cut = min(x for x in (died, trip) if x is not None) if (died or trip) else None
    before = [t for t in mine if cut is not None and t <= cut]
    after = [t for t in mine if restarted is not None and t >= restarted]
    back = first(lambda k, w, v: k.endswith(dev) and w == "status" and v == "online",
                 after=restarted or 0.0) if restarted is not None else None
    last_ok = round(before[-1], 2) if before else None
    first_new = round(after[0], 2) if after else None
    return {"last_job_before_fault_s": last_ok, "breaker_trip_s": trip, "worker_died_s": died,
            "worker_restarted_s": restarted, "device_online_again_s": back,
            "first_job_after_restart_s": first_new,
            "recovery_s": (round(first_new - last_ok, 2)
                           if first_new is not None and last_ok is not None else None),
            "events": [(round(t - t0, 2), k, w, v) for t, k, w, v in timeline
                       if k.endswith(dev) or w in ("alive", "restarts")][:60]}


async def _wait_workers(url: str, n: int, timeout: float = 900) -> None:
    import aiohttp
    t_end = time.time() + timeout
    async with aiohttp.ClientSession() as s:
        while time.time() < t_end:
            try:
                async with s.get(url + "/v1/dashboard") as r:
                    d = await r.json()
                    if d.get("workers_online", 0) >= n:
                        return
            except Exception:
                pass
            _log("waiting for workers to register")
            await asyncio.sleep(5.0)
    raise TimeoutError("workers never came online")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["queue", "embed", "mixed"])
    ap.add_argument("--store", default=os.environ.get("LMX_STORE", "memory"))
    ap.add_argument("--jobs", type=int, default=2000)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--capacity", type=int, default=16)
    ap.add_argument("--gpu", type=int, default=0)
    ap.add_argument("--gpus", default="0")
    ap.add_argument("--model", default="nomic-embed-text")
    ap.add_argument("--chat-model", default="llama-3-8b")
    ap.add_argument("--concurrency", type=int, default=32)
    ap.add_argument("--requests", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--chars", type=int, default=1024)
    ap.add_argument("--embed-every", type=int, default=4)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--sync-every", type=int, default=0,
                    help="mixed: every k-th request is a sync /v1/chat/completions call")
    ap.add_argument("--replicas-per-gpu", type=int, default=1,
                    help="mixed: workers per GPU (1-GPU rehearsal of a multi-GPU node)")
    ap.add_argument("--fault", default="", help="mixed: LMX_FAULT spec for the targeted worker")
    ap.add_argument("--fault-device", default="", help="mixed: device-id suffix, e.g. gpu0.r1")
    ap.add_argument("--fault-lives", type=int, default=0,
                    help="mixed: inject only in the first N lives of the faulty worker (0 = all)")
    ap.add_argument("--await-recovery", type=float, default=0.0,
                    help="mixed: after the load, wait up to S seconds for every worker to be "
                         "alive and its device online again; reports recovered_after_s")
    ap.add_argument("--cpu", action="store_true", help="mixed: CPU engines (plumbing)")
    ap.add_argument("--runs", type=int, default=1,
                    help="mixed: repeat the whole run (fresh serve each time) and report the "
                         "median jobs/s with the spread; pair with a fixed fault schedule "
                         "(--fault gpu_error@N) so runs differ only in performance")
    a = ap.parse_args(argv)
    fn = {"queue": bench_queue, "embed": bench_embed, "mixed": bench_mixed}[a.what]
    if a.what == "mixed" and a.runs > 1:
        runs = [fn(a) for _ in range(a.runs)]
        rates = sorted(r["jobs_per_s"] for r in runs)
        med = sorted(runs, key=lambda r: r["jobs_per_s"])[len(runs) // 2]
        out = dict(med, runs=a.runs, jobs_per_s_runs=[r["jobs_per_s"] for r in runs],
                   jobs_per_s_median=med["jobs_per_s"],
                   spread_pct=round((rates[-1] - rates[0]) / med["jobs_per_s"] * 100, 1))
        print(json.dumps(out), flush=True)
        return
    print(json.dumps(fn(a)), flush=True)


if __name__ == "__main__":
    main()
