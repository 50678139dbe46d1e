"""Command line: ``python -m llm_mcp_amd <command>``.

  serve      core (HTTP :8080 + gRPC :9090) + one GPU worker process per GPU
             (or one TP group), the production launcher on an 8x MI355X node
  core       the core only (attach to already running workers with --engine)
  worker     one GPU worker (see worker/main.py)
  mcp        MCP tool server (stdio; --http for streamable HTTP)
  bridge     HTTP bridge (:3333)
  telemetry  alert loop
  build      compile the native extensions in-tree
  config     print every environment setting (typed, defaults, current)

The parent of ``serve`` never initialises HIP: GPUs are enumerated from sysfs
and every worker is spawned before anything touches a device.
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
import subprocess
import sys

log = logging.getLogger("lmx")


def _gpu_list(spec: str) -> list[int]:
    out = []
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


async def run_core(args, specs, procs=()):
    from aiohttp import web

    from .api.core import CoreState, create_core_app
    from .api.serve import attach_engines
    from .devices import rocm_enum
    from .rpc.server import start_grpc

    addrs = {}
    for s in specs:
        dev = s.get("device", "gpu0")
        if dev.startswith("gpu"):
            dev = rocm_enum.device_id(int(dev[3:]))
            s["device"] = dev
        addrs[dev] = "unix:" + s["path"]
    st = CoreState(engine_addrs=addrs)
    st.engines_ready = not specs
    app = create_core_app(st)
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    host, port = args.http.rsplit(":", 1)
    await web.TCPSite(runner, host or "0.0.0.0", int(port)).start()
    grpc_srv, _ = await start_grpc(st, args.grpc)
    log.info("core up: http %s grpc %s, %d engines", args.http, args.grpc, len(specs))
    if specs:
        await attach_engines(st, specs)
        await asyncio.to_thread(st.discovery.run)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        loop.add_signal_handler(sig, stop.set)

    async def watch():
        while not stop.is_set():
            for p in procs:
                if p.poll() is not None:
                    log.error("worker pid %d exited with %s", p.pid, p.returncode)
                    await asyncio.to_thread(st.discovery.run)
            await asyncio.sleep(5)

    w = asyncio.create_task(watch())
    await stop.wait()
    w.cancel()
    await grpc_srv.stop(5)   # drain gRPC too (the reference only shut down HTTP)
    await runner.cleanup()


def cmd_serve(args):
    from .devices import rocm_enum
    gpus = _gpu_list(args.gpus) if args.gpus else [g.index for g in rocm_enum.enumerate_gpus()]
    if not gpus:
        sys.exit("no GPUs found (set --gpus or LMX_FAKE_GPUS)")
    embed_gpus = set(_gpu_list(args.embed_gpus)) if args.embed_gpus else set(gpus)
    host = rocm_enum.host_id()
    procs, specs = [], []
    env = dict(os.environ)
    env.setdefault("CORE_GRPC_ADDR", "127.0.0.1" + args.grpc[args.grpc.rfind(":"):])
    env.setdefault("CORE_HTTP_URL", "http://127.0.0.1" + args.http[args.http.rfind(":"):])
    if args.tp > 1:
        groups = [gpus[i:i + args.tp] for i in range(0, len(gpus), args.tp)]
        for grp in groups:
            sock = f"/tmp/lmx-{host}-tp{args.tp}-gpu{grp[0]}.sock"
            e = dict(env, HIP_VISIBLE_DEVICES=",".join(map(str, grp)))
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={len(grp)}", "--master-addr", "127.0.0.1",
                   "--master-port", str(29500 + grp[0]), "-m", "llm_mcp_amd.worker.main",
                   "--tp", str(args.tp), "--chat-model", args.chat_model, "--socket", sock]
            procs.append(subprocess.Popen(cmd, env=e))
            specs.append({"model": args.chat_model, "path": sock,
                          "device": f"{host}:tp{args.tp}:gpu{grp[0]}-{grp[-1]}"})
    else:
        for g in gpus:
            sock = f"/tmp/lmx-{host}-gpu{g}.sock"
            cmd = [sys.executable, "-m", "llm_mcp_amd.worker.main", "--gpu", str(g),
                   "--chat-model", args.chat_model, "--socket", sock,
                   "--max-num-seqs", str(args.max_num_seqs)]
            if args.embed_model and g in embed_gpus:
                cmd += ["--embed-model", args.embed_model]
            procs.append(subprocess.Popen(cmd, env=env))
            if args.chat_model:
                specs.append({"model": args.chat_model, "path": sock, "device": f"gpu{g}"})
            if args.embed_model and g in embed_gpus:
                specs.append({"model": args.embed_model, "path": sock, "device": f"gpu{g}"})
    try:
        asyncio.run(run_core(args, specs, procs))
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()


def cmd_core(args):
    from .api.serve import parse_engine_spec
    asyncio.run(run_core(args, [parse_engine_spec(s) for s in args.engine]))


def main(argv=None):
    logging.basicConfig(level=os.environ.get("LOG_LEVEL", "INFO"),
                        format='{"ts":"%(asctime)s","level":"%(levelname)s",'
                               '"component":"%(name)s","msg":"%(message)s"}')
    ap = argparse.ArgumentParser(prog="llm_mcp_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in ("serve", "core"):
        p = sub.add_parser(name)
        p.add_argument("--http", default=os.environ.get("CORE_HTTP_ADDR", ":8080"))
        p.add_argument("--grpc", default=os.environ.get("CORE_GRPC_ADDR", ":9090"))
        if name == "serve":
            p.add_argument("--gpus", default=os.environ.get("LMX_GPUS", ""))
            p.add_argument("--chat-model", default=os.environ.get("LMX_CHAT_MODEL", "llama-3-8b"))
            p.add_argument("--embed-model", default=os.environ.get("LMX_EMBED_MODEL", ""))
            p.add_argument("--embed-gpus", default="")
            p.add_argument("--tp", type=int, default=int(os.environ.get("LMX_TP", "1")))
            p.add_argument("--max-num-seqs", type=int, default=256)
        else:
            p.add_argument("--engine", action="append", default=[])
    sub.add_parser("worker", add_help=False)
    sub.add_parser("mcp", add_help=False)
    sub.add_parser("bridge")
    sub.add_parser("telemetry")
    sub.add_parser("build")
    sub.add_parser("config")
    args, rest = ap.parse_known_args(argv)
    if args.cmd != "config":
        from . import settings
        settings.validate()
    if args.cmd == "serve":
        cmd_serve(args)
    elif args.cmd == "core":
        cmd_core(args)
    elif args.cmd == "worker":
        from .worker.main import main as wm
        wm(rest)
    elif args.cmd == "mcp":
        from .mcp.server import main as mm
        sys.argv = [sys.argv[0]] + rest
        mm()
    elif args.cmd == "bridge":
        from .mcp.bridge import main as bm
        bm()
    elif args.cmd == "telemetry":
        from .telemetry.alerts import main as tm
        tm()
    elif args.cmd == "config":
        from .settings import table
        print(table())
    elif args.cmd == "build":
        from .build import build_all
        build_all(force="--force" in rest, verbose=True)


if __name__ == "__main__":
    main()
