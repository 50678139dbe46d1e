#!/usr/bin/env python3
"""Headline benchmark: tokens/s + p50 TTFT via /v1/chat/completions,
Llama-3-8B (bf16, random-init weights, synthetic prompts) on N MI355X.

One process per GPU (torchrun / torch.distributed.run, RCCL process group):
every rank serves a full data-parallel Llama-3-8B replica behind its own
OpenAI-compatible HTTP server (aiohttp, SSE streaming, in-process engine with
the gfx950 HIP kernels) and drives it with its own load-generator subprocess
(started before the GPU is initialised).  One "step" = one wave of
``--concurrency`` concurrent streaming chat requests per GPU, each with a
``--prompt-len``-token synthetic prompt and ``--max-tokens`` generated tokens
(ignore_eos).  W untimed warmup waves, then exactly K timed waves bracketed by
barrier + device synchronize on both sides; the job value is the total
completion tokens of all ranks divided by the slowest rank's time.

Prints ONE JSON line on rank 0 (driver contract).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import threading
import time

BASELINE = None  # the reference publishes no throughput number (BASELINE.json "published": {})


def log(msg: str) -> None:
    print(f"[bench r{os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--concurrency", type=int, default=256, help="concurrent streams per GPU")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--temperature", type=float, default=0.8)
    ap.add_argument("--top-p", type=float, default=0.95)
    ap.add_argument("--port-base", type=int, default=18080)
    ap.add_argument("--max-batched-tokens", type=int, default=16384)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--inproc", action="store_true",
                    help="serve HTTP from the GPU process (default: separate API process)")
    ap.add_argument("--rehearse-on-one-gpu", action="store_true",
                    help="multi-rank rehearsal on a 1-GPU box: every rank uses device 0, gloo "
                         "process group, a fixed KV budget (never used for reported numbers)")
    a = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    port = a.port_base + local_rank
    url = f"http://127.0.0.1:{port}"
    sock = f"/tmp/lmx-bench-{os.getpid()}-{local_rank}.sock"

    # children first: no process is started after this one touches the GPU
    api_proc = None
    if not a.inproc:
        api_proc = subprocess.Popen(
            [sys.executable, "-m", "llm_mcp_amd.api.serve", "--port", str(port),
             "--engine", f"{a.model}=unix:{sock},device=gpu{local_rank}"],
            stdout=subprocess.DEVNULL)
    client = subprocess.Popen(
        [sys.executable, "-m", "llm_mcp_amd.bench.loadgen", "--serve-stdin", "--url", url,
         "--model", a.model, "--concurrency", str(a.concurrency), "--prompt-len",
         str(a.prompt_len), "--max-tokens", str(a.max_tokens), "--temperature",
         str(a.temperature), "--top-p", str(a.top_p)],
        stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)

    import torch
    import torch.distributed as dist

    from llm_mcp_amd import ops
    from llm_mcp_amd.api.app import ServingState, make_app
    from llm_mcp_amd.api.registry import LocalModel, ModelRegistry
    from llm_mcp_amd.engine.async_engine import AsyncEngine
    from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine
    from llm_mcp_amd.models.tokenizer import for_model
    from llm_mcp_amd.utils.metrics import Metrics

    gpu = 0 if a.rehearse_on_one_gpu else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if a.rehearse_on_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    ops.native()  # fail loudly if the HIP kernels are missing

    t_init = time.time()
    ecfg = EngineConfig(model=a.model, max_num_seqs=max(a.concurrency, 1),
                        max_batched_tokens=a.max_batched_tokens,
                        max_model_len=min(8192, a.prompt_len + a.max_tokens + 64),
                        use_graphs=not a.no_graphs, seed=rank,
                        kv_cache_gb=24 if a.rehearse_on_one_gpu else None)
    engine = LLMEngine(ecfg, device=dev)
    log(f"engine ready in {time.time() - t_init:.1f}s: {engine.num_blocks} KV blocks, "
        f"{len(engine.graphs)} decode graphs, weights {engine.model.weight_bytes() / 1e9:.1f} GB")
    loop = None
    if a.inproc:
        aeng = AsyncEngine(engine)
        reg = ModelRegistry()
        reg.add(LocalModel(a.model, "chat", f"gpu{local_rank}", aeng, for_model(engine.cfg),
                           engine.cfg, max_model_len=engine.max_model_len,
                           capacity=ecfg.max_num_seqs))
        state = ServingState(reg, Metrics())
        state.register_routes = lambda app: app.router.add_get(
            "/ready", lambda r: __import__("aiohttp").web.json_response({"ready": True}))

        from aiohttp import web
        loop = asyncio.new_event_loop()
        started = threading.Event()

        def serve():
            asyncio.set_event_loop(loop)
            runner = web.AppRunner(make_app(state), access_log=None)
            loop.run_until_complete(runner.setup())
            loop.run_until_complete(web.TCPSite(runner, "127.0.0.1", port).start())
            aeng.start(loop)
            started.set()
            loop.run_forever()

        threading.Thread(target=serve, daemon=True, name="http").start()
        started.wait()
    else:
        from llm_mcp_amd.engine.ipc import EngineServer
        server = EngineServer(engine, sock, info={
            "kind": "chat", "model": a.model, "device_id": f"gpu{local_rank}",
            "max_model_len": engine.max_model_len, "capacity": ecfg.max_num_seqs})
        server.start()
    ready = json.loads(client.stdout.readline())
    if not ready.get("ready"):
        raise RuntimeError("load generator could not reach the server")

    def run_wave():
        client.stdin.write("run\n")
        client.stdin.flush()
        line = client.stdout.readline()
        if not line:
            raise RuntimeError("load generator exited")
        return json.loads(line)

    def barrier():
        if world > 1:
            dist.barrier()

    for w in range(a.warmup):
        r = run_wave()
        log(f"warmup {w}: {r['tokens']} tok in {r['elapsed']:.2f}s ({r['tok_s']:.0f} tok/s), "
            f"ttft p50 {r['ttft_p50'] * 1e3:.0f} ms")
    for k in engine.stats:
        engine.stats[k] = type(engine.stats[k])(0)
    engine.ttft_samples.clear()
    import psutil
    procs = {"engine": psutil.Process(), "loadgen": psutil.Process(client.pid)}
    if api_proc is not None:
        procs["api"] = psutil.Process(api_proc.pid)
    cpu0 = {k: sum(p.cpu_times()[:2]) for k, p in procs.items()}
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    results = []
    for k in range(a.steps):
        r = run_wave()
        results.append(r)
        log(f"step {k}: {r['tokens']} tok in {r['elapsed']:.2f}s ({r['tok_s']:.0f} tok/s), "
            f"ttft p50 {r['ttft_p50'] * 1e3:.0f} ms, itl p50 {r['itl_p50'] * 1e3:.1f} ms")
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0

    log("process CPU utilisation over the timed waves: " + ", ".join(
        f"{k} {(sum(p.cpu_times()[:2]) - cpu0[k]) / elapsed * 100:.0f}%" for k, p in procs.items()))
    st = engine.stats
    ns = max(1, st["steps"])
    log("engine host phases (ms/step avg over all steps): " + ", ".join(
        f"{k[2:]} {st[k] / ns * 1e3:.3f}" for k in st if k.startswith("t_")) +
        f"; steps {st['steps']} graph {st['graph_steps']}, decode step "
        f"{st['decode_step_s'] / max(1, st['graph_steps']) * 1e3:.2f} ms")
    if engine.ttft_samples:
        from llm_mcp_amd.bench.loadgen import percentile as _pct
        et = [f - a for a, f in engine.ttft_samples]
        log(f"engine-side TTFT (submit -> first token emitted) p50 {_pct(et, 50) * 1e3:.0f} ms, "
            f"p95 {_pct(et, 95) * 1e3:.0f} ms over {len(et)} requests")
    tokens = sum(r["tokens"] for r in results)
    ttfts = [t for r in results for t in r["ttfts"]]
    mine = {"tokens": tokens, "elapsed": elapsed, "ttfts": ttfts,
            "itl": [r["itl_p50"] for r in results]}
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, mine)
    else:
        allr = [mine]
    client.stdin.write("quit\n")
    client.stdin.flush()
    if rank == 0:
        from llm_mcp_amd.bench.loadgen import percentile
        tot = sum(x["tokens"] for x in allr)
        slow = max(x["elapsed"] for x in allr)
        all_ttft = [t for x in allr for t in x["ttfts"]]
        value = tot / slow
        st = engine.stats
        out = {
            "metric": "tokens/sec + p50 TTFT via /v1/chat/completions, Llama-3-8B at 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "tokens/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(slow / a.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None if BASELINE is None else round(value / BASELINE, 3),
            "dtype": "bf16",
            "data": "synthetic prompts, random-init weights",
            "ttft_p50_ms": round(percentile(all_ttft, 50) * 1e3, 1),
            "ttft_p95_ms": round(percentile(all_ttft, 95) * 1e3, 1),
            "itl_p50_ms": round(percentile([i for x in allr for i in x["itl"]], 50) * 1e3, 2),
            "config": {"model": a.model, "global_batch": a.concurrency * world,
                       "seq_len": a.prompt_len + a.max_tokens, "prompt_len": a.prompt_len,
                       "max_tokens": a.max_tokens, "parallelism": f"dp{world}",
                       "endpoint": "/v1/chat/completions stream=true",
                       "serving": "in-process" if a.inproc else "api process + engine process (unix socket)",
                       "sampling": {"temperature": a.temperature, "top_p": a.top_p},
                       "engine_steps": st["steps"], "graph_steps": st["graph_steps"]},
        }
        print(json.dumps(out), flush=True)
    barrier()
    try:
        client.wait(timeout=30)
    except Exception:
        client.kill()
    engine.stop()
    if loop is not None:
        loop.call_soon_threadsafe(loop.stop)
    if api_proc is not None:
        api_proc.terminate()
        try:
            api_proc.wait(timeout=10)
        except Exception:
            api_proc.kill()
        if os.path.exists(sock):
            os.unlink(sock)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
