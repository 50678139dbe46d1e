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


def plan_placement(gpus: list[int], chat_model: str = "", embed_model: str = "",
                   embed_gpus: list[int] | None = None, tp: int = 1,
                   registry: str = "") -> list[dict]:
    """Which worker process serves what (SURVEY §5.6 ``LMX_MODEL_REGISTRY``).

    Without a registry every GPU gets ``chat_model`` (TP groups of ``tp``
    consecutive GPUs when tp > 1) and ``embed_model`` on ``embed_gpus``.  A
    registry places models per GPU set, entries separated by ``;``::

        GPUS:MODEL          single-GPU chat engines on each listed GPU
        GPUS:tpN:MODEL      TP=N groups over the listed GPUs (N consecutive each)
        GPUS:embed:MODEL    embedding engine on each listed GPU

    e.g. ``0-3:llama-3-8b;4-7:tp4:llama-3-70b;0-3:embed:nomic-embed-text``.
    A GPU holds at most one chat engine (or one TP rank) and one embedder;
    TP ranks carry no embedder.  Returns launch entries
    ``{"gpus": [...], "tp": n, "chat": model | "", "embed": model | ""}``.
    """
    if not registry:
        if tp > 1:
            if len(gpus) % tp:
                raise ValueError(f"{len(gpus)} GPUs do not split into TP={tp} groups")
            return [{"gpus": gpus[i:i + tp], "tp": tp, "chat": chat_model, "embed": ""}
                    for i in range(0, len(gpus), tp)]
        eg = set(gpus if embed_gpus is None else embed_gpus)
        return [{"gpus": [g], "tp": 1, "chat": chat_model,
                 "embed": embed_model if embed_model and g in eg else ""} for g in gpus]
    single: dict[int, dict] = {}
    groups: list[dict] = []
    in_group: set[int] = set()
    for raw in registry.split(";"):
        ent = raw.strip()
        if not ent:
            continue
        parts = ent.split(":")
        if len(parts) == 2:
            gspec, role, model = parts[0], "chat", parts[1]
        elif len(parts) == 3:
            gspec, role, model = parts
        else:
            raise ValueError(f"bad registry entry {ent!r}")
        model = model.strip()
        role = role.strip().lower()
        sel = _gpu_list(gspec)
        if not sel or not model:
            raise ValueError(f"bad registry entry {ent!r}")
        unknown = [g for g in sel if g not in gpus]
        if unknown:
            raise ValueError(f"registry entry {ent!r}: GPUs {unknown} are not served")
        if role.startswith("tp"):
            n = int(role[2:])
            if n < 1 or len(sel) % n:
                raise ValueError(f"registry entry {ent!r}: {len(sel)} GPUs do not split into "
                                 f"TP={n} groups")
            for i in range(0, len(sel), n):
                grp = sel[i:i + n]
                for g in grp:
                    if g in in_group or (g in single and single[g]["chat"]) or \
                            (n > 1 and g in single):
                        raise ValueError(f"GPU {g} is placed twice")
                if n == 1:
                    single.setdefault(grp[0], {"gpus": grp, "tp": 1, "chat": "", "embed": ""})
                    single[grp[0]]["chat"] = model
                else:
                    in_group.update(grp)
                    groups.append({"gpus": grp, "tp": n, "chat": model, "embed": ""})
            continue
        if role not in ("chat", "embed"):
            raise ValueError(f"registry entry {ent!r}: role must be tpN, chat or embed")
        for g in sel:
            if g in in_group:
                raise ValueError(f"GPU {g} is a TP rank and cannot host {model}")
            w = single.setdefault(g, {"gpus": [g], "tp": 1, "chat": "", "embed": ""})
            if w[role]:
                raise ValueError(f"GPU {g} already has a {role} model ({w[role]})")
            w[role] = model
    return [single[g] for g in sorted(single)] + groups


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
            idx, _, rep = dev[3:].partition(".")
            dev = rocm_enum.device_id(int(idx)) + (f".{rep}" if rep else "")
            s["device"] = dev
        addrs[dev] = "unix:" + s["path"]
    st = CoreState(engine_addrs=addrs)
    st.engines_ready = not specs
    app = create_core_app(st)
    if isinstance(procs, Supervisor):
        from .api.helpers import write_json

        async def workers(request):
            """Supervised GPU worker processes: pid, alive, restarts."""
            return write_json(200, {"workers": procs.status()})
        app.router.add_get("/v1/debug/workers", workers)
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
            died = await asyncio.to_thread(procs.poll) if isinstance(procs, Supervisor) else []
            if died:
                # replicas of a dead worker already left the registry (its engine
                # link closed, api/serve.py); discovery marks its devices' state
                await asyncio.to_thread(st.discovery.run)
            await asyncio.sleep(SUPERVISE_TICK_S)

    w = asyncio.create_task(watch())
    await stop.wait()
    w.cancel()
    for t in getattr(st, "engine_links", []):
        t.cancel()
    await grpc_srv.stop(5)   # drain gRPC too (the reference only shut down HTTP)
    await runner.cleanup()


SUPERVISE_TICK_S = 1.0


class Supervisor:
    """Keeps the GPU worker processes of ``serve`` alive.

    Each worker is a child process started from a command line; the parent
    (which never initialises HIP) starts a FRESH child when one exits -- never
    a re-exec of a process that touched the GPU -- with exponential backoff
    (``LMX_RESTART_BACKOFF_S`` doubling up to ``LMX_RESTART_MAX_S``; reset
    after a worker stayed up for a minute).  The reference gets the same
    behaviour from its process manager (compose.yml:117,133,149
    ``restart: unless-stopped``, k8s Deployments)."""

    def __init__(self, restart: bool = True):
        self.restart = restart
        self.entries: list[dict] = []
        self.base = float(os.environ.get("LMX_RESTART_BACKOFF_S", "1"))
        self.cap = float(os.environ.get("LMX_RESTART_MAX_S", "60"))

    def spawn(self, cmd: list[str], env: dict, name: str) -> subprocess.Popen:
        import time
        p = subprocess.Popen(cmd, env=dict(env, LMX_WORKER_LIFE="1"))
        self.entries.append({"cmd": cmd, "env": env, "name": name, "proc": p,
                             "started": time.time(), "backoff": self.base,
                             "restart_at": None, "restarts": 0})
        return p

    def poll(self) -> list[str]:
        """Reap exited workers and (re)start the ones whose backoff expired.
        Returns the names of workers found dead on this tick."""
        import time
        now, died = time.time(), []
        for e in self.entries:
            p = e["proc"]
            if p is not None and p.poll() is not None:
                log.error("worker %s (pid %d) exited with %s", e["name"], p.pid, p.returncode)
                died.append(e["name"])
                if now - e["started"] > 60:
                    e["backoff"] = self.base
                e["proc"] = None
                e["restart_at"] = now + e["backoff"] if self.restart else None
                e["backoff"] = min(self.cap, e["backoff"] * 2)
            if e["proc"] is None and e["restart_at"] is not None and now >= e["restart_at"]:
                # LMX_WORKER_LIFE: 1-based life of this worker slot (fault
                # schedules may target the first lives only: LMX_FAULT_LIVES)
                e["proc"] = subprocess.Popen(e["cmd"], env=dict(
                    e["env"], LMX_WORKER_LIFE=str(e["restarts"] + 2)))
                e["started"], e["restart_at"] = now, None
                e["restarts"] += 1
                log.warning("worker %s restarted (pid %d, restart #%d)", e["name"],
                            e["proc"].pid, e["restarts"])
        return died

    def status(self) -> list[dict]:
        return [{"name": e["name"], "pid": e["proc"].pid if e["proc"] is not None else None,
                 "alive": e["proc"] is not None and e["proc"].poll() is None,
                 "restarts": e["restarts"]} for e in self.entries]

    def __iter__(self):
        return iter([e["proc"] for e in self.entries if e["proc"] is not None])

    def __len__(self):
        return len(self.entries)

    def stop(self, timeout: float | None = None) -> None:
        if timeout is None:
            timeout = float(os.environ.get("LMX_STOP_GRACE_S", "20"))
        for e in self.entries:
            e["restart_at"] = None
        live = [e["proc"] for e in self.entries if e["proc"] is not None]
        for p in live:
            p.terminate()
        for p in live:
            try:
                p.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                p.kill()


def cmd_serve(args):
    from .devices import rocm_enum
    gpus = _gpu_list(args.gpus) if args.gpus else [g.index for g in rocm_enum.enumerate_gpus()]
    if not gpus:
        sys.exit("no GPUs found (set --gpus or LMX_FAKE_GPUS)")
    try:
        plan = plan_placement(gpus, args.chat_model, args.embed_model,
                              _gpu_list(args.embed_gpus) if args.embed_gpus else None,
                              args.tp, args.registry)
    except ValueError as e:
        sys.exit(f"placement: {e}")
    host = rocm_enum.host_id()
    sup = Supervisor(restart=not args.no_restart)
    specs = []
    env = dict(os.environ)
    env.setdefault("CORE_GRPC_ADDR", "127.0.0.1" + args.grpc[args.grpc.rfind(":"):])
    env.setdefault("CORE_HTTP_URL", "http://127.0.0.1" + args.http[args.http.rfind(":"):])
    sock_dir = args.socket_dir or "/tmp"
    extra = ["--cpu"] if args.cpu else []
    if args.weights:       # real checkpoint for the chat model (each TP rank loads its shard)
        extra += ["--weights", args.weights]
    plan = [dict(w, replica=k) for w in plan for k in range(max(1, args.replicas_per_gpu))
            if k == 0 or w["tp"] == 1]
    for w in plan:
        grp, tp = w["gpus"], w["tp"]
        if tp > 1:
            sock = os.path.join(sock_dir, f"lmx-{host}-tp{tp}-gpu{grp[0]}.sock")
            e = dict(env, HIP_VISIBLE_DEVICES=",".join(map(str, grp)))
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                   f"--nproc-per-node={len(grp)}", "--master-addr", "127.0.0.1",
                   "--master-port", str(29500 + grp[0]), "-m", "llm_mcp_amd.worker.main",
                   "--tp", str(tp), "--chat-model", w["chat"], "--socket", sock,
                   "--max-num-seqs", str(args.max_num_seqs)] + extra
            sup.spawn(cmd, e, f"tp{tp}:gpu{grp[0]}-{grp[-1]}")
            specs.append({"model": w["chat"], "path": sock,
                          "device": f"{host}:tp{tp}:gpu{grp[0]}-{grp[-1]}"})
            continue
        g, k = grp[0], w["replica"]
        name = f"gpu{g}" + (f".r{k}" if k else "")
        sock = os.path.join(sock_dir, f"lmx-{host}-{name}.sock")
        cmd = [sys.executable, "-m", "llm_mcp_amd.worker.main", "--gpu", str(g),
               "--chat-model", w["chat"], "--socket", sock,
               "--max-num-seqs", str(args.max_num_seqs)] + extra
        if k:
            cmd += ["--replica", str(k)]
        if args.kv_fraction:
            cmd += ["--kv-fraction", str(args.kv_fraction)]
        if w["embed"]:
            cmd += ["--embed-model", w["embed"]]
        sup.spawn(cmd, env, name)
        for m in (w["chat"], w["embed"]):
            if m:
                specs.append({"model": m, "path": sock, "device": name})
    try:
        asyncio.run(run_core(args, specs, sup))
    finally:
        sup.stop()


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
            p.add_argument("--weights", default=os.environ.get("LMX_WEIGHTS", ""),
                           help="safetensors dir of the chat model's real weights")
            p.add_argument("--max-num-seqs", type=int,
                           default=int(os.environ.get("LMX_MAX_BATCH", "256")))
            p.add_argument("--registry", default=os.environ.get("LMX_MODEL_REGISTRY", ""),
                           help="per-GPU placement, e.g. '0-3:llama-3-8b;4-7:tp4:llama-3-70b;"
                                "0-3:embed:nomic-embed-text' (overrides --chat-model/--tp)")
            p.add_argument("--no-restart", action="store_true",
                           help="do not restart GPU workers that exit")
            p.add_argument("--socket-dir", default=os.environ.get("LMX_SOCKET_DIR", ""))
            p.add_argument("--cpu", action="store_true",
                           help="workers run their engines on the CPU (tests / plumbing)")
            p.add_argument("--replicas-per-gpu", type=int, default=1,
                           help="single-GPU workers per GPU (1-GPU rehearsals of a multi-GPU "
                                "node; device ids gpuN.rk)")
            p.add_argument("--kv-fraction", type=float, default=0.0,
                           help="KV cache share of free HBM per worker (0: worker default)")
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
