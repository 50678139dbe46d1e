#!/usr/bin/env python3
"""Headline benchmark: tokens/s + p50 TTFT via /v1/chat/completions,
Llama-3-8B (bf16, random-init weights, synthetic prompts) on N MI355X.

Topology -- the product's serving path, one front door for the whole node:

  rank r (one process per GPU, torch.distributed.run; the bench starts the
          ranks itself when run without a launcher and --gpus > 1)
      one Llama-3-8B engine on cuda:r (continuous batching, the gfx950 HIP
      kernels, captured decode graphs) served on an engine socket
      (engine/ipc.py) -- the GPU worker of ``python -m llm_mcp_amd serve``
  rank 0, before it touches the GPU, also starts
      * the FRONT DOOR: A API processes (api/serve.py) sharing ONE port via
        SO_REUSEPORT, each attached to all N engines and routing every
        stream with ModelRegistry.select (least loaded healthy replica)
      * L load-generator processes (bench/loadgen.py) that together keep
        N x C streaming chat requests in flight against that one port

One "step" = one wave of N x ``--concurrency`` concurrent streaming chat
requests (``--prompt-len``-char synthetic prompt, ``--max-tokens`` generated,
ignore_eos).  W untimed warmup waves, then exactly K timed waves bracketed by
a barrier + ``torch.cuda.synchronize()`` on both sides on every rank; the
elapsed time is the max over ranks and the value is all completion tokens
streamed to the clients divided by it (weak scaling: C streams per GPU).

``--tp T`` (BASELINE config 4, e.g. Llama-3-70B at T = 8): the N ranks form
N / T tensor-parallel groups of T consecutive ranks (RCCL subgroups); each
group's rank 0 is the engine behind the front door, its followers execute
the leader's plans on their weight shards (parallel/tp_worker.py), and
``--concurrency`` counts streams per engine.

Prints ONE JSON line on rank 0 (driver contract).  ``--gpus`` must equal the
launcher's WORLD_SIZE (a mismatch exits non-zero).  ``--rehearse-on-one-gpu``
runs every rank on cuda:0 (a plumbing rehearsal on a 1-GPU box; its line is
flagged and is never an N-GPU number).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

BASELINE = None  # the reference publishes no throughput number (BASELINE.json "published": {})
METRIC = "tokens/sec + p50 TTFT via /v1/chat/completions, Llama-3-8B at 1/2/4/8 MI355X"
HERE = os.path.dirname(os.path.abspath(__file__))


def log(msg: str) -> None:
    print(f"[bench r{os.environ.get('RANK', '0')}] {msg}", file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--concurrency", type=int, default=256,
                    help="concurrent streams per engine (per GPU at --tp 1)")
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree: N/T engines of T GPUs each")
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--temperature", type=float, default=0.8)
    ap.add_argument("--top-p", type=float, default=0.95)
    ap.add_argument("--max-batched-tokens", type=int, default=None,
                    help="tokens per engine step (default: the engine's, LMX_MAX_BATCHED_TOKENS)")
    ap.add_argument("--mixed-prefill-tokens", type=int, default=None,
                    help="prompt tokens per mixed step (default: the engine's, "
                         "LMX_MIXED_PREFILL_TOKENS; 0 = no cap)")
    ap.add_argument("--api-procs", type=int, default=0,
                    help="front-door API processes on the shared port (0: two per engine, "
                         "at most 16)")
    ap.add_argument("--loadgen-procs", type=int, default=0,
                    help="load-generator processes (0: two per engine, at most 16)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--load", choices=("waves", "closed", "poisson"), default="waves",
                    help="waves (the headline: K synchronized waves of C streams per GPU), "
                         "closed (C streams per GPU at constant concurrency, each client sending "
                         "its next request when its stream ends, for --duration seconds after "
                         "--closed-warmup seconds) or poisson (open loop: --rate requests/s per "
                         "GPU arriving as a Poisson process); the latter two are separate "
                         "records, never the headline")
    ap.add_argument("--rate", type=float, default=60.0,
                    help="--load poisson: arrivals per second per GPU")
    ap.add_argument("--duration", type=float, default=30.0)
    ap.add_argument("--closed-warmup", type=float, default=10.0)
    ap.add_argument("--cpu", action="store_true",
                    help="plumbing mode for tests: every rank runs its engine on the CPU (gloo; "
                         "use a tiny model such as tiny-llama); never a reported number")
    ap.add_argument("--rehearse-on-one-gpu", action="store_true",
                    help="multi-rank rehearsal on a 1-GPU box: every rank uses device 0 with a "
                         "fixed KV budget (never used for reported numbers)")
    return ap.parse_args(argv)


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(a) -> None:
    """--gpus N > 1 without a launcher: start N ranks as CHILD processes
    (nothing here has touched the GPU) and exit with their status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    log("launching " + " ".join(cmd[2:]))
    sys.exit(subprocess.call(cmd))


def start_front_door(a, world: int, tag: str, socks: list[str]):
    """Rank 0, before any HIP call: the API processes (one shared port) and
    the load generators.  Returns (api procs, loadgen procs, url, ready files).
    ``socks``: one engine socket per engine (per TP group)."""
    port = free_port()
    url = f"http://127.0.0.1:{port}"
    n_eng = len(socks)
    # two API processes and two load generators per engine: the wave's request
    # burst and its SSE chunks spread over more event loops (1x1 / 2x2 / 4x4 on
    # one GPU: 16,709 / 16,770 / 16,788 tok/s, client - engine TTFT 27 / 16 / 9 ms)
    n_api = a.api_procs or min(16, 2 * n_eng)
    n_lg = a.loadgen_procs or min(16, 2 * n_eng)
    engines = []
    for g, s in enumerate(socks):
        dev = f"gpu{g}" if a.tp == 1 else f"tp{a.tp}:gpu{g * a.tp}-{(g + 1) * a.tp - 1}"
        engines += ["--engine", f"{a.model}=unix:{s},device={dev}"]
    env = dict(os.environ, LOG_LEVEL=os.environ.get("LMX_BENCH_API_LOG", "WARNING"))
    # node-wide in-flight counts: the API processes balance on them together,
    # so no engine receives more streams than its slots (api/shared_load.py)
    load_file = f"/dev/shm/lmx-bench-{tag}.load"
    if os.path.exists(load_file):
        os.unlink(load_file)
    apis, ready_files = [], [load_file]     # ready files + the load file: all removed at exit
    for i in range(n_api):
        rf = f"/tmp/lmx-bench-{tag}-api{i}.ready"
        if os.path.exists(rf):
            os.unlink(rf)
        ready_files.append(rf)
        apis.append(subprocess.Popen(
            [sys.executable, "-m", "llm_mcp_amd.api.serve", "--port", str(port),
             "--reuse-port", "--ready-file", rf, "--shared-load", load_file,
             "--api-index", str(i), "--api-count", str(n_api)] + engines,
            cwd=HERE, env=env, stdout=subprocess.DEVNULL))
    total = a.concurrency * n_eng
    per = [total // n_lg + (1 if i < total % n_lg else 0) for i in range(n_lg)]
    lgs = []
    for i, c in enumerate(per):
        lgs.append(subprocess.Popen(
            [sys.executable, "-m", "llm_mcp_amd.bench.loadgen", "--serve-stdin", "--url", url,
             "--model", a.model, "--concurrency", str(c), "--prompt-len", str(a.prompt_len),
             "--max-tokens", str(a.max_tokens), "--temperature", str(a.temperature),
             "--top-p", str(a.top_p), "--seed-base", str(i + 1)],
            cwd=HERE, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True))
    return apis, lgs, url, ready_files


def main() -> None:
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        self_launch(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if a.tp < 1 or world % a.tp:
        sys.exit(f"bench.py: --tp {a.tp} does not divide --gpus {world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_eng, grp, grank = world // a.tp, rank // a.tp, rank % a.tp
    # all ranks of one launch share their parent (the torchrun agent)
    tag = str(os.getppid() if "WORLD_SIZE" in os.environ and world > 1 else os.getpid())
    socks = [f"/tmp/lmx-bench-{tag}-{g}.sock" for g in range(n_eng)]

    apis, lgs, ready_files = [], [], []
    if rank == 0:
        # children first: no process is started after this one touches the GPU
        apis, lgs, url, ready_files = start_front_door(a, world, tag, socks)

    import torch
    import torch.distributed as dist

    from llm_mcp_amd import ops
    from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine
    from llm_mcp_amd.engine.ipc import EngineServer

    gpu = 0 if a.rehearse_on_one_gpu else local_rank
    if a.cpu:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)

    def sync():
        if not a.cpu:
            torch.cuda.synchronize()
    if world > 1:
        # control plane only (barriers, timing, per-GPU stats): data-parallel
        # serving exchanges no tensors between GPUs
        import datetime
        os.environ.setdefault("GLOO_SOCKET_IFNAME", "lo")
        dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=60))
    if not a.cpu:
        ops.native()  # fail loudly if the HIP kernels are missing
    tpctx = None
    if a.tp > 1:
        # every rank creates every group's subgroups, in the same order
        from llm_mcp_amd.models.llama import TPContext
        for g in range(n_eng):
            ranks = list(range(g * a.tp, (g + 1) * a.tp))
            # one GPU per rank: RCCL over xGMI; a one-GPU rehearsal cannot put
            # several ranks of one communicator on one device: gloo + the
            # peer-memory all-reduce kernel (decode sizes)
            tg = dist.new_group(ranks, backend="gloo" if (a.rehearse_on_one_gpu or a.cpu)
                                else "nccl")
            cg = dist.new_group(ranks, backend="gloo")
            if g == grp:
                tpctx = TPContext(grank, a.tp, tg, cpu_group=cg)

    t_init = time.time()
    # the serving defaults `serve` ships (engine.EngineConfig) unless overridden
    knobs = {k: v for k, v in (("max_batched_tokens", a.max_batched_tokens),
                               ("mixed_prefill_tokens", a.mixed_prefill_tokens)) if v is not None}
    ecfg = EngineConfig(model=a.model, max_num_seqs=max(a.concurrency, 1), **knobs,
                        max_model_len=min(8192, a.prompt_len + a.max_tokens + 64),
                        use_graphs=not a.no_graphs, seed=rank,
                        # rehearsal: every rank shares cuda:0's 288 GB
                        kv_cache_gb=(max(4, min(24, 128 // world)) if a.rehearse_on_one_gpu
                                     else None) if not a.cpu else 0.05)
    follower = None
    if tpctx is None:
        engine = LLMEngine(ecfg, device=dev)
    else:
        import threading

        from llm_mcp_amd.parallel.tp_worker import build_tp_engine
        engine = build_tp_engine(ecfg, dev, tpctx, f"bench-{tag}-g{grp}")
        if grank:
            # followers execute the leader's plans until it releases them
            follower = threading.Thread(target=engine.run_follower, name="tp-follower",
                                        daemon=True)
            follower.start()
    log(f"engine ready on {dev} in {time.time() - t_init:.1f}s: {engine.num_blocks} KV "
        f"blocks, {len(engine.graphs)} decode graphs, "
        f"weights {engine.model.weight_bytes() / 1e9:.1f} GB "
        f"({engine.model.weight_bytes(copies=True) / 1e9:.1f} GB with packed copies)"
        + (f" (TP rank {grank}/{a.tp} of engine {grp})" if a.tp > 1 else ""))
    server = None
    if grank == 0:
        server = EngineServer(engine, socks[grp], info={
            "kind": "chat", "model": a.model,
            "device_id": f"gpu{rank}" if a.tp == 1 else f"tp{a.tp}:gpu{rank}-{rank + a.tp - 1}",
            "max_model_len": engine.max_model_len, "capacity": ecfg.max_num_seqs})
        server.start()

    def barrier():
        if world > 1:
            dist.barrier()

    def waves(n: int, label: str) -> list[dict]:
        out = []
        for k in range(n):
            t_w = time.time()
            for p in lgs:
                p.stdin.write("run\n")
                p.stdin.flush()
            parts = []
            for p in lgs:
                line = p.stdout.readline()
                if not line:
                    raise RuntimeError("load generator exited")
                parts.append(json.loads(line))
            r = {"tokens": sum(x["tokens"] for x in parts),
                 "elapsed": max(x["elapsed"] for x in parts),
                 "requests": sum(x["requests"] for x in parts),
                 "ttfts": [t for x in parts for t in x["ttfts"]],
                 "itls": [t for x in parts for t in x["itls"]],
                 "gaps": [sum(c) for c in zip(*(x["gaps"] for x in parts))]}
            out.append(r)
            from llm_mcp_amd.bench.loadgen import percentile as pct
            log(f"{label} {k}: {r['requests']} streams, {r['tokens']} tok in {r['elapsed']:.2f}s "
                f"({r['tokens'] / r['elapsed']:.0f} tok/s), ttft p50 "
                f"{pct(r['ttfts'], 50) * 1e3:.0f} ms, itl p50 {pct(r['itls'], 50) * 1e3:.1f} ms")
            if engine.step_trace is not None:
                # LMX_STEP_TRACE=1: this wave's eager steps (launch ms after the
                # wave started: rows / decode rows / prefill tokens / waiting)
                tr = [x for x in engine.step_trace if x[0] >= t_w]
                log(f"{label} {k} eager steps: " + " ".join(
                    f"{(x[0] - t_w) * 1e3:.0f}ms:T{x[1]}/d{x[2]}/p{x[3]}/w{x[4]}" for x in tr))
        return out

    import psutil
    if rank == 0:
        t_wait = time.time()
        while not all(os.path.exists(f) for f in ready_files):
            if any(p.poll() is not None for p in apis):
                raise RuntimeError("a front-door API process exited")
            if time.time() - t_wait > 1800:
                raise RuntimeError("front door never attached every engine")
            time.sleep(0.2)
        for p in lgs:
            ready = json.loads(p.stdout.readline())
            if not ready.get("ready"):
                raise RuntimeError("load generator could not reach the front door")
        log(f"front door up: {len(apis)} API processes on {url}, {len(lgs)} load generators, "
            f"{a.concurrency * n_eng} streams per wave over {n_eng} engines")
    barrier()
    if rank == 0:
        waves(a.warmup, "warmup")
    barrier()

    for k in engine.stats:
        engine.stats[k] = type(engine.stats[k])(0)
    engine.ttft_samples.clear()
    procs = {"engine": [psutil.Process()]}
    if rank == 0:
        procs["api"] = [psutil.Process(p.pid) for p in apis]
        procs["loadgen"] = [psutil.Process(p.pid) for p in lgs]

    def cpu_s(ps):
        return sum(sum(p.cpu_times()[:2]) for p in ps)
    cpu0 = {k: cpu_s(v) for k, v in procs.items()}

    if a.load in ("closed", "poisson"):
        closed(a, rank, world, n_eng, lgs, barrier, sync, engine.ecfg, engine)
        shutdown(a, world, lgs, apis, server, ready_files, engine, follower)
        return

    # clocks / power / temperature around the timed waves (rank 0, every card
    # of the node): a slower box is told apart from a regression
    clocks = {}
    if rank == 0 and not a.cpu:
        from llm_mcp_amd.devices.rocm_enum import gpu_clock_snapshot
        clocks["start"] = gpu_clock_snapshot()
    barrier()
    sync()
    t0 = time.perf_counter()
    results = waves(a.steps, "step") if rank == 0 else []
    barrier()           # the other ranks serve until rank 0's waves are done
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if rank == 0 and not a.cpu:
        clocks["end"] = gpu_clock_snapshot()

    cpu = {k: (cpu_s(v) - cpu0[k]) / elapsed * 100 for k, v in procs.items()}
    st = engine.stats
    ns = max(1, st["steps"])
    log("process CPU % over the timed waves: " + ", ".join(f"{k} {v:.0f}%" for k, v in cpu.items()))
    log("engine host phases (ms/step avg over all steps): " + ", ".join(
        f"{k[2:]} {st[k] / ns * 1e3:.3f}" for k in st if k.startswith("t_")) +
        f"; steps {st['steps']} graph {st['graph_steps']}, decode step "
        f"{st['decode_step_s'] / max(1, st['graph_steps']) * 1e3:.2f} ms (host: " + ", ".join(
            f"{k[2:]} {st[k] / max(1, st['graph_steps']) * 1e3:.3f}" for k in st
            if k.startswith("g_")) + ")")
    # engine-side TTFT: request arrival at the engine -> first token handed to
    # the IPC link (the client-side figure adds the front door and SSE path)
    e_ttft = sorted(now - arr for arr, now in list(engine.ttft_samples))
    e_ttft_p50 = e_ttft[len(e_ttft) // 2] * 1e3 if e_ttft else None
    mine = {"rank": rank, "elapsed": elapsed, "gen_tokens": int(st["generated_tokens"]),
            "engine_ttft_p50_ms": e_ttft_p50,
            "finished": int(st["finished"]), "steps": int(st["steps"]),
            "graph_steps": int(st["graph_steps"]),
            "decode_ms": st["decode_step_s"] / max(1, st["graph_steps"]) * 1e3,
            "engine_cpu_pct": cpu["engine"]}
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, mine)
    else:
        allr = [mine]

    for p in lgs:
        p.stdin.write("quit\n")
        p.stdin.flush()
    if rank == 0:
        from llm_mcp_amd.bench.loadgen import percentile
        slow = max(x["elapsed"] for x in allr)
        tokens = sum(r["tokens"] for r in results)
        ttfts = [t for r in results for t in r["ttfts"]]
        itls = [t for r in results for t in r["itls"]]
        value = tokens / slow
        # tokens are generated by the engines (TP leaders): one entry per engine
        per_gpu = [round(x["gen_tokens"] / slow, 1) for x in allr if x["rank"] % a.tp == 0]
        nz = [v for v in per_gpu if v > 0]
        out = {
            "metric": METRIC,
            "value": round(value, 1), "unit": "tokens/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(slow / a.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None if BASELINE is None else round(value / BASELINE, 3),
            "dtype": "bf16",
            "data": "synthetic prompts, random-init weights",
            "ttft_p50_ms": round(percentile(ttfts, 50) * 1e3, 1),
            "ttft_p95_ms": round(percentile(ttfts, 95) * 1e3, 1),
            "itl_p50_ms": round(percentile(itls, 50) * 1e3, 2),
            "itl_p95_ms": round(percentile(itls, 95) * 1e3, 2),
            "itl_p99_ms": round(percentile(itls, 99) * 1e3, 2),
            **gap_percentiles(results),
            "per_gpu_tok_s": per_gpu,
            "gpu_balance_max_over_min": round(max(nz) / min(nz), 3) if nz else None,
            "decode_step_ms": [round(x["decode_ms"], 2) for x in allr],
            "engine_ttft_p50_ms": [None if x["engine_ttft_p50_ms"] is None else
                                   round(x["engine_ttft_p50_ms"], 1) for x in allr],
            "front_door_cpu_pct": round(cpu.get("api", 0.0), 1),
            "loadgen_cpu_pct": round(cpu.get("loadgen", 0.0), 1),
            "engine_cpu_pct": [round(x["engine_cpu_pct"], 1) for x in allr],
            "gpu_clocks": clocks or None,
            "config": {"model": a.model, "global_batch": a.concurrency * n_eng,
                       "seq_len": a.prompt_len + a.max_tokens, "prompt_len": a.prompt_len,
                       "max_tokens": a.max_tokens,
                       "parallelism": f"dp{world}" if a.tp == 1 else
                       (f"tp{a.tp}" if n_eng == 1 else f"dp{n_eng}xtp{a.tp}"),
                       "endpoint": "/v1/chat/completions stream=true",
                       "serving": f"{n_eng} engine(s) of {a.tp} GPU(s) behind one front door: "
                                  f"{len(apis)} "
                                  f"API process(es) on one SO_REUSEPORT port, replica "
                                  f"selection per stream; {len(lgs)} load generator(s)",
                       "sampling": {"temperature": a.temperature, "top_p": a.top_p},
                       "engine": {"lookahead_stepping": bool(engine.lookahead),
                                  "decode_graph_buckets": len(engine.graphs),
                                  "kv_pages": "K [BS][D] token-major, V [BS/4][D][4] key-quad",
                                  "max_batched_tokens": ecfg.max_batched_tokens,
                                  "mixed_prefill_tokens": ecfg.mixed_prefill_tokens,
                                  "mixed_min_decodes": engine.ecfg.mixed_min_decodes,
                                  "mixed_later_steps": engine.ecfg.mixed_later_steps},
                       "tp_group": None if a.tp == 1 else {
                           "collectives": "gloo (one-GPU rehearsal)" if (a.rehearse_on_one_gpu or a.cpu)
                           else "nccl (RCCL)",
                           "peer_memory_allreduce_allgather": tpctx is not None and
                           tpctx.peer is not None,
                           "startup_selftest": getattr(engine, "tp_selftest", None),
                           "lookahead": bool(engine.lookahead)},
                       "engine_steps": sum(x["steps"] for x in allr),
                       "graph_steps": sum(x["graph_steps"] for x in allr)},
        }
        if a.rehearse_on_one_gpu:
            out["rehearsal_one_gpu"] = True
            out["config"]["parallelism"] += " (rehearsal: every rank on cuda:0, NOT an "\
                                            f"{world}-GPU number)"
        if a.cpu:
            out["cpu_plumbing"] = True
            out["config"]["parallelism"] += " (CPU plumbing test, NOT a GPU number)"
        print(json.dumps(out), flush=True)
    barrier()
    shutdown(a, world, lgs, apis, server, ready_files, engine, follower)


def shutdown(a, world, lgs, apis, server, ready_files, engine=None, follower=None) -> None:
    for p in lgs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    if server is not None:
        server.stop()
    if engine is not None and a.tp > 1:
        if follower is None:
            engine.release_followers()
        else:
            follower.join(timeout=60)
        if engine.chan is not None:
            engine.chan.close()
    for p in apis:
        p.terminate()
    for p in apis:
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()
    for f in ready_files:
        if os.path.exists(f):
            os.unlink(f)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def gap_percentiles(parts) -> dict:
    """Per-token inter-arrival gap p50 / p95 / p99 (ms) from the load
    generators' merged histograms (bench/loadgen.py GAP_BINS)."""
    from llm_mcp_amd.bench.loadgen import GAP_BINS, hist_percentile
    h = [0] * GAP_BINS
    for x in parts:
        for i, c in enumerate(x.get("gaps") or ()):
            h[i] += c
    return {f"token_gap_p{q}_ms": round(hist_percentile(h, q) * 1e3, 2) for q in (50, 95, 99)}


def closed(a, rank, world, n_eng, lgs, barrier, sync, ecfg, engine=None) -> None:
    """--load closed / poisson: one steady-load window through the same front
    door; prints its own JSON line (metric tagged "closed loop" / "poisson")."""
    from llm_mcp_amd.bench.loadgen import percentile
    barrier()
    sync()
    parts = []
    if rank == 0:
        for p in lgs:
            if a.load == "poisson":
                # the engine's rate split over its load generators
                per = a.rate * n_eng / len(lgs)
                p.stdin.write(f"open {per} {a.closed_warmup} {a.duration}\n")
            else:
                p.stdin.write(f"closed {a.closed_warmup} {a.duration}\n")
            p.stdin.flush()
        # a heartbeat line a minute, so a long window (--duration 600: a soak run)
        # is not mistaken for a hung process by whoever watches the log
        done = threading.Event()

        def beat():
            t0 = time.time()
            g0 = engine.stats["generated_tokens"] if engine is not None else 0
            while not done.wait(60.0):
                extra = ""
                if engine is not None:      # this rank's engine, over the last minute
                    g = engine.stats["generated_tokens"]
                    extra = f"; engine r0 {(g - g0) / 60.0:,.0f} generated tok/s"
                    g0 = g
                log(f"{a.load} window: {time.time() - t0:.0f} s of "
                    f"{a.closed_warmup + a.duration:g} s{extra}")
        threading.Thread(target=beat, daemon=True).start()
        for p in lgs:
            parts.append(json.loads(p.stdout.readline()))
        done.set()
    barrier()
    if rank == 0:
        tok = sum(x["tokens"] for x in parts)
        ttfts = [t for x in parts for t in x["ttfts"]]
        itls = [t for x in parts for t in x["itls"]]
        tag = "closed loop" if a.load == "closed" else "poisson arrivals"
        load = (f"closed loop: {a.concurrency} streams per GPU, next request on stream end"
                if a.load == "closed" else
                f"open loop: Poisson arrivals at {a.rate:g} requests/s per GPU "
                f"({sum(x.get('arrivals', 0) for x in parts)} arrivals)")
        out = {"metric": METRIC + f" [{tag}]", "value": round(tok / a.duration, 1),
               "unit": "tokens/s", "n_gpus": world, "duration_s": a.duration,
               "requests": sum(x["requests"] for x in parts), "dtype": "bf16",
               "data": "synthetic prompts, random-init weights",
               "ttft_p50_ms": round(percentile(ttfts, 50) * 1e3, 1),
               "ttft_p95_ms": round(percentile(ttfts, 95) * 1e3, 1),
               "ttft_p99_ms": round(percentile(ttfts, 99) * 1e3, 1),
               "itl_p50_ms": round(percentile(itls, 50) * 1e3, 2),
               "itl_p95_ms": round(percentile(itls, 95) * 1e3, 2),
               "itl_p99_ms": round(percentile(itls, 99) * 1e3, 2),
               **gap_percentiles(parts),
               "config": {"model": a.model, "concurrency": a.concurrency * n_eng,
                          "prompt_len": a.prompt_len, "max_tokens": a.max_tokens,
                          "max_batched_tokens": ecfg.max_batched_tokens,
                          "mixed_prefill_tokens": ecfg.mixed_prefill_tokens,
                          "mixed_later_steps": ecfg.mixed_later_steps,
                          "load": f"{load}, {a.closed_warmup:g} s warm-up, "
                                  f"{a.duration:g} s window",
                          "sampling": {"temperature": a.temperature, "top_p": a.top_p}}}
        if a.rehearse_on_one_gpu:
            out["rehearsal_one_gpu"] = True
        print(json.dumps(out), flush=True)
        for p in lgs:
            p.stdin.write("quit\n")
            p.stdin.flush()
    barrier()


if __name__ == "__main__":
    main()
