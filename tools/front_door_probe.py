"""Front-door overhead probe (CPU only, no model): the API processes and the
load generator of bench.py against a synthetic engine that answers every
request with one token per simulated step.

The synthetic engine records when each request reaches it, so the probe
separates the two costs the client's TTFT carries on top of the engine's:
the spread of request arrivals at the start of a wave (HTTP parse, chat
template, tokenisation, IPC submit in the API processes) and the token path
back (IPC event -> SSE chunk -> client).

    python tools/front_door_probe.py [--streams 256] [--api-procs 1] [--step-ms 10]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llm_mcp_amd.bench.loadgen import percentile  # noqa: E402
from llm_mcp_amd.engine.engine import TokenEvent  # noqa: E402
from llm_mcp_amd.engine.ipc import EngineServer  # noqa: E402


class _Sched:
    num_running = 0
    num_waiting = 0
    kv_usage = 0.0
    kv_free_blocks = 1 << 20


class SyntheticEngine:
    """Duck-typed stand-in for LLMEngine behind EngineServer: every running
    request gets one token per step (token ``tok``), the first at the first
    step after its arrival."""

    def __init__(self, step_ms: float, tok: int, first_ms: float = 0.0):
        self._ids = itertools.count(1)
        self.sched = _Sched()
        self.stats: dict = {}
        self.event_sink = None
        self.step_s = step_ms / 1e3
        self.first_s = first_ms / 1e3      # simulated prefill: no token before this
        self.tok = tok
        self._new: list = []
        self._run: list = []
        self._lock = threading.Lock()
        self._stop = False
        self.arrivals: list[float] = []

    def submit(self, req):
        now = time.perf_counter()
        req.arrival = now
        with self._lock:
            self.arrivals.append(now)
            self._new.append(req)

    def abort(self, rid):
        with self._lock:
            self._run = [r for r in self._run if r.id != rid]

    def start(self):
        threading.Thread(target=self._loop, daemon=True, name="synthetic-engine").start()

    def stop(self):
        self._stop = True

    def _loop(self):
        nxt = time.perf_counter()
        while not self._stop:
            nxt += self.step_s
            time.sleep(max(0.0, nxt - time.perf_counter()))
            now = time.perf_counter()
            with self._lock:
                due = [r for r in self._new if now - r.arrival >= self.first_s]
                self._new = [r for r in self._new if now - r.arrival < self.first_s]
                self._run += due
                run = list(self._run)
            evs = []
            for r in run:
                r.num_generated += 1
                fin = "length" if r.num_generated >= r.params.max_tokens else None
                evs.append(TokenEvent(r, self.tok, 0.0, fin))
            with self._lock:
                self._run = [r for r in self._run if r.num_generated < r.params.max_tokens]
                self.sched.num_running = len(self._run)
            if evs and self.event_sink is not None:
                self.event_sink(evs)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--api-procs", type=int, default=1)
    ap.add_argument("--step-ms", type=float, default=10.0)
    ap.add_argument("--first-ms", type=float, default=0.0,
                    help="simulated prefill: a request's first token no earlier than this")
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--waves", type=int, default=3)
    ap.add_argument("--loadgens", type=int, default=1)
    ap.add_argument("--profile-api", default="", help="cProfile output path of API process 0")
    a = ap.parse_args()
    model = "llama-3-8b"
    from llm_mcp_amd.models import config as mc
    from llm_mcp_amd.models.tokenizer import for_model
    tok = for_model(mc.resolve(model), None).encode("a")[-1]
    eng = SyntheticEngine(a.step_ms, tok, a.first_ms)
    tmp = tempfile.mkdtemp(prefix="lmx-fdp-")
    sock = os.path.join(tmp, "engine.sock")
    srv = EngineServer(eng, sock, info={"kind": "chat", "model": model, "device_id": "gpu0",
                                        "max_model_len": 8192, "capacity": a.streams})
    srv.start()
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    url = f"http://127.0.0.1:{port}"
    load_file = f"/dev/shm/lmx-fdp-{os.getpid()}.load"   # as bench.py: tmpfs
    apis, ready = [], []
    env = dict(os.environ, LOG_LEVEL="WARNING")
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for i in range(a.api_procs):
        rf = os.path.join(tmp, f"api{i}.ready")
        ready.append(rf)
        prof = ["-m", "cProfile", "-o", a.profile_api] if a.profile_api and i == 0 else []
        apis.append(subprocess.Popen(
            [sys.executable] + prof + ["-m", "llm_mcp_amd.api.serve", "--port", str(port), "--reuse-port",
             "--ready-file", rf, "--shared-load", load_file, "--api-index", str(i),
             "--api-count", str(a.api_procs), "--engine", f"{model}=unix:{sock},device=gpu0"],
            cwd=here, env=env, stdout=subprocess.DEVNULL))
    per = [a.streams // a.loadgens + (1 if i < a.streams % a.loadgens else 0)
           for i in range(a.loadgens)]
    lgs = [subprocess.Popen(
        [sys.executable, "-m", "llm_mcp_amd.bench.loadgen", "--serve-stdin", "--url", url,
         "--model", model, "--concurrency", str(c), "--prompt-len", str(a.prompt_len),
         "--max-tokens", str(a.max_tokens), "--seed-base", str(i + 1)],
        cwd=here, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
        for i, c in enumerate(per)]
    try:
        t0 = time.time()
        while not all(os.path.exists(f) for f in ready):
            if time.time() - t0 > 120:
                raise RuntimeError("API processes never became ready")
            time.sleep(0.1)
        for lg in lgs:
            if not json.loads(lg.stdout.readline()).get("ready"):
                raise RuntimeError("load generator could not reach the front door")
        for w in range(a.waves):
            eng.arrivals.clear()
            for lg in lgs:
                lg.stdin.write("run\n")
                lg.stdin.flush()
            parts = [json.loads(lg.stdout.readline()) for lg in lgs]
            r = {"requests": sum(x["requests"] for x in parts),
                 "tokens": sum(x["tokens"] for x in parts),
                 "elapsed": max(x["elapsed"] for x in parts),
                 "ttfts": [t for x in parts for t in x["ttfts"]]}
            arr = sorted(eng.arrivals)
            spread = [(t - arr[0]) * 1e3 for t in arr]
            print(json.dumps({
                "wave": w, "streams": r["requests"], "api_procs": a.api_procs,
                "loadgens": a.loadgens,
                "step_ms": a.step_ms, "first_ms": a.first_ms, "tok_s": round(r["tokens"] / r["elapsed"]),
                "client_ttft_p50_ms": round(percentile(r["ttfts"], 50) * 1e3, 1),
                "client_ttft_p95_ms": round(percentile(r["ttfts"], 95) * 1e3, 1),
                "arrival_spread_p50_ms": round(percentile(spread, 50), 1),
                "arrival_spread_max_ms": round(spread[-1], 1) if spread else 0.0}), flush=True)
    finally:
        for lg in lgs:
            lg.stdin.write("quit\n")
            lg.stdin.flush()
        for lg in lgs:
            lg.wait(timeout=30)
        for p in apis:
            p.terminate()
        for p in apis:
            p.wait(timeout=30)
        srv.stop()
        if os.path.exists(load_file):
            os.unlink(load_file)


if __name__ == "__main__":
    main()
