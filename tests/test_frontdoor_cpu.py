"""Multi-GPU serving topology on the CPU: N engine worker processes behind one
front door (tiny-llama engines on the CPU stand in for per-GPU workers).

* streams through ONE API port are spread over the engines by
  ModelRegistry.select (bench.py's topology);
* two API processes can share the port (SO_REUSEPORT) and balance on shared
  node-wide in-flight counts (api/shared_load.py);
* ``serve`` supervises its workers: a worker killed mid-wave fails only its
  own streams, new streams go to the survivors, and a fresh worker process
  re-joins (reference compose.yml ``restart:
  unless-stopped``).
"""
import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

import aiohttp
import pytest

from llm_mcp_amd.bench.loadgen import wave
from llm_mcp_amd.engine.ipc import EngineClient

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, LOG_LEVEL="WARNING", OMP_NUM_THREADS="1")


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(sock: str, gpu: int, seqs: int = 16) -> subprocess.Popen:
    return subprocess.Popen(
        [sys.executable, "-m", "llm_mcp_amd.worker.main", "--cpu", "--gpu", str(gpu),
         "--chat-model", "tiny-llama", "--socket", sock, "--no-jobs",
         "--max-num-seqs", str(seqs), "--max-batched-tokens", "512", "--max-model-len", "512"],
        cwd=ROOT, env=ENV)


async def _wait_ready(url: str, replicas: int, timeout: float = 120) -> dict:
    t_end = time.time() + timeout
    async with aiohttp.ClientSession() as s:
        while time.time() < t_end:
            try:
                async with s.get(url + "/ready") as r:
                    body = await r.json()
                    if r.status == 200 and body.get("replicas", replicas) >= replicas:
                        return body
            except (aiohttp.ClientError, json.JSONDecodeError):
                pass
            await asyncio.sleep(0.2)
    raise TimeoutError(f"{url} never reported {replicas} replicas")


async def _finished(sock: str) -> int:
    c = EngineClient(sock)
    await c.connect(timeout=30)
    try:
        return int((await c.info(timeout=10))["stats"]["finished"])
    finally:
        await c.close()


def _stop(procs):
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            p.kill()


@pytest.mark.timeout(300)
def test_front_door_balances_streams_over_engines():
    n, streams = 4, 64
    d = tempfile.mkdtemp()
    socks = [os.path.join(d, f"e{i}.sock") for i in range(n)]
    procs = [_worker(s, i) for i, s in enumerate(socks)]
    port = _port()
    url = f"http://127.0.0.1:{port}"
    eng = []
    for i, s in enumerate(socks):
        eng += ["--engine", f"tiny-llama=unix:{s},device=gpu{i}"]
    # two API processes on one port balancing on shared node-wide counts, as
    # bench.py runs the front door
    load = os.path.join("/dev/shm", f"lmx-test-{os.getpid()}.load")
    apis = [subprocess.Popen([sys.executable, "-m", "llm_mcp_amd.api.serve", "--port",
                              str(port), "--reuse-port", "--shared-load", load,
                              "--api-index", str(i), "--api-count", "2"] + eng, cwd=ROOT, env=ENV)
            for i in range(2)]
    try:
        async def go():
            await _wait_ready(url, n)
            await asyncio.sleep(1.0)    # let the second API process attach too
            await _wait_ready(url, n)
            before = [await _finished(s) for s in socks]
            r = await wave(url, "tiny-llama", streams, 48, 8, 0.8, 0.95, 7)
            assert r["requests"] == streams and r["tokens"] == streams * 8
            after = [await _finished(s) for s in socks]
            return [b - a for a, b in zip(before, after)]
        per = asyncio.new_event_loop().run_until_complete(go())
        assert sum(per) == streams, per
        # both processes select on the shared counts: as even as one process
        assert max(per) - min(per) <= 0.1 * streams / n + 1, per
    finally:
        _stop(apis + procs)
        if os.path.exists(load):
            os.unlink(load)


@pytest.mark.timeout(300)
def test_single_api_process_even_split():
    n, streams = 4, 64
    d = tempfile.mkdtemp()
    socks = [os.path.join(d, f"e{i}.sock") for i in range(n)]
    procs = [_worker(s, i) for i, s in enumerate(socks)]
    port = _port()
    url = f"http://127.0.0.1:{port}"
    eng = []
    for i, s in enumerate(socks):
        eng += ["--engine", f"tiny-llama=unix:{s},device=gpu{i}"]
    api = subprocess.Popen([sys.executable, "-m", "llm_mcp_amd.api.serve", "--port", str(port)]
                           + eng, cwd=ROOT, env=ENV)
    try:
        async def go():
            await _wait_ready(url, n)
            before = [await _finished(s) for s in socks]
            await wave(url, "tiny-llama", streams, 48, 8, 0.8, 0.95, 3)
            after = [await _finished(s) for s in socks]
            return [b - a for a, b in zip(before, after)]
        per = asyncio.new_event_loop().run_until_complete(go())
        assert sum(per) == streams
        assert max(per) - min(per) <= 0.1 * streams / n + 1, per   # within +-10 %
    finally:
        _stop([api] + procs)


@pytest.mark.timeout(300)
def test_serve_restarts_a_dead_worker_and_routes_around_it():
    n = 3
    d = tempfile.mkdtemp()
    http, grpc = _port(), _port()
    url = f"http://127.0.0.1:{http}"
    env = dict(ENV, LMX_FAKE_GPUS=str(n), LMX_RESTART_BACKOFF_S="0.5", LMX_STORE="memory",
               DISCOVERY_INTERVAL="0")
    core = subprocess.Popen(
        [sys.executable, "-m", "llm_mcp_amd", "serve", "--cpu", "--gpus", f"0-{n - 1}",
         "--chat-model", "tiny-llama", "--max-num-seqs", "16", "--socket-dir", d,
         "--http", f"127.0.0.1:{http}", "--grpc", f"127.0.0.1:{grpc}"],
        cwd=ROOT, env=env, start_new_session=True)
    import psutil
    try:
        async def go():
            await _wait_ready(url, n, timeout=180)
            kids = [c for c in psutil.Process(core.pid).children()
                    if "llm_mcp_amd.worker.main" in " ".join(c.cmdline())]
            assert len(kids) == n, [c.cmdline() for c in kids]
            victim = kids[0]
            # long streams in flight on every engine, then kill one worker
            task = asyncio.ensure_future(_many(url, 24, 400))
            await asyncio.sleep(1.5)
            victim.send_signal(signal.SIGKILL)
            res = await task
            ok = [r for r in res if r == "ok"]
            bad = [r for r in res if r != "ok"]
            # only the victim's share failed, and it failed cleanly
            assert ok and len(bad) <= 24 // n + 2, res
            assert all(r in ("error", "http-502") for r in bad), bad
            # new streams while the replacement starts: all served by survivors
            res2 = await _many(url, 12, 4)
            assert all(r == "ok" for r in res2), res2
            # the supervisor started a fresh process; it re-joins the registry
            body = await _wait_ready(url, n, timeout=180)
            assert body["replicas"] == n
            kids2 = [c for c in psutil.Process(core.pid).children()
                     if "llm_mcp_amd.worker.main" in " ".join(c.cmdline())]
            assert len(kids2) == n and victim.pid not in {c.pid for c in kids2}
        asyncio.new_event_loop().run_until_complete(go())
    finally:
        try:
            os.killpg(core.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        try:
            core.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(core.pid, signal.SIGKILL)


async def _many(url: str, n: int, max_tokens: int) -> list[str]:
    async def one(s, i):
        body = {"model": "tiny-llama", "messages": [{"role": "user", "content": f"q{i}"}],
                "stream": True, "max_tokens": max_tokens, "ignore_eos": True,
                "temperature": 0.7}
        fin = None
        async with s.post(url + "/v1/chat/completions", json=body) as r:
            if r.status != 200:
                return f"http-{r.status}"
            async for line in r.content:
                if line.startswith(b"data: ") and line[6:].strip() != b"[DONE]":
                    ch = json.loads(line[6:]).get("choices") or []
                    if ch and ch[0].get("finish_reason"):
                        fin = ch[0]["finish_reason"]
        return "ok" if fin in ("length", "stop") else (fin or "none")
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=240)) as s:
        return await asyncio.gather(*[one(s, i) for i in range(n)])


@pytest.mark.timeout(400)
def test_config5_mixed_load_with_a_faulty_replica():
    """BASELINE config 5 in miniature (CPU engines): two workers on one
    device, injected HIP faults on one of them.  Every async job completes
    (failed attempts requeue to the healthy worker), sync chat errors stay
    bounded, the faulty worker is restarted by the supervisor, and the
    breaker of the faulty device trips."""
    import json as _json
    env = dict(ENV, LMX_FAKE_GPUS="1")
    out = subprocess.run(
        [sys.executable, "-m", "llm_mcp_amd.bench.serving_bench", "mixed", "--cpu", "--gpus",
         "0", "--replicas-per-gpu", "2", "--fault", "gpu_error:0.03", "--fault-device",
         "gpu0.r1", "--chat-model", "tiny-llama", "--model", "tiny-nomic", "--jobs", "400",
         "--concurrency", "8", "--sync-every", "2", "--max-tokens", "16", "--chars", "64"],
        cwd=ROOT, env=env, capture_output=True, text=True, timeout=380)
    assert out.returncode == 0, out.stderr[-3000:]
    r = _json.loads(out.stdout.strip().splitlines()[-1])
    assert r["error_rate"] == 0.0, r                         # async jobs all done
    assert r["sync_chat"]["ok"] >= 0.8 * (r["sync_chat"]["ok"] + r["sync_chat"]["error"]), r
    faulty = next(w for w in r["workers"] if w["name"] == "gpu0.r1")
    healthy = next(w for w in r["workers"] if w["name"] == "gpu0")
    assert faulty["restarts"] >= 1 and healthy["restarts"] == 0, r["workers"]
    dev = next(d for d in r["circuit_states_seen"] if d.endswith("gpu0.r1"))
    assert "degraded" in r["circuit_states_seen"][dev], r["circuit_states_seen"]
    # the fault -> recovery phases on the bench's own clock
    rec = r["recovery"]
    assert rec["breaker_trip_s"] is not None and rec["worker_restarted_s"] is not None, rec
    assert rec["worker_died_s"] <= rec["worker_restarted_s"], rec
