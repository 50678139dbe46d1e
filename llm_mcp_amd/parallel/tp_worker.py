"""Tensor-parallel serving group (Llama-3-70B TP=8 over xGMI).

Launched by ``python -m llm_mcp_amd serve --tp N`` as one
``torch.distributed.run`` group per N GPUs (one process per GPU, RCCL
process group).  Rank 0 is the group's *leader*: it owns the continuous-
batching scheduler, the engine <-> API socket and the job agent, exactly like
a single-GPU worker, and publishes every step's plan on the shared-memory
mailbox (plan_channel.py).  Ranks 1..N-1 are *followers*: they execute the
same forward on their weight shard.  Per layer the group does two RCCL
all-reduces (after the O and down projections, X1/X2) and one all-gather of
the vocab-split logits per step (X3); the decode graphs capture those
collectives together with the kernels.

The reference has no model parallelism at all; its nearest
notion is "one Ollama per host".
"""
from __future__ import annotations

import logging
import os
import time

import torch
import torch.distributed as dist

from ..models.llama import TPContext
from .plan_channel import LeaderLost, PlanChannel, mailbox_path

log = logging.getLogger("lmx.tp")


def init_group(device: torch.device | str | None = None) -> TPContext:
    """Join the torchrun-launched group (env:// rendezvous, 127.0.0.1)."""
    rank = int(os.environ.get("RANK", "0"))
    size = int(os.environ.get("WORLD_SIZE", "1"))
    if size == 1:
        return TPContext()
    if not dist.is_initialized():
        dev = torch.device(device) if device is not None else None
        if dev is not None and dev.type == "cuda":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    return TPContext(rank, size, dist.group.WORLD)


class GroupSelfTestError(RuntimeError):
    pass


def group_self_test(tp: TPContext, device: torch.device, timeout_s: float | None = None) -> dict:
    """Startup check of the TP group's device collectives (RCCL on GPUs):
    an all-reduce and an all-gather of seeded values, compared exactly with
    what every rank can compute on the host.  A wrong result raises
    ``GroupSelfTestError``; a collective that does not return within
    ``timeout_s`` (LMX_TP_SELFTEST_S, default 180) ends the process with a
    clear message and exit code 3 instead of hanging the whole launch (a
    stuck RCCL call cannot be interrupted from Python)."""
    if tp.size < 2:
        return {}
    import threading
    timeout_s = float(os.environ.get("LMX_TP_SELFTEST_S", "180")) if timeout_s is None \
        else timeout_s
    done = threading.Event()

    def watchdog():
        if not done.wait(timeout_s):
            msg = (f"TP group self-test: rank {tp.rank}/{tp.size} waited {timeout_s:.0f} s for "
                   f"the {dist.get_backend(tp.group)} collectives on {device}; a rank is missing "
                   "or the interconnect is down -- exiting instead of hanging")
            log.error(msg)
            print(msg, flush=True)
            os._exit(3)
    threading.Thread(target=watchdog, name="tp-selftest-watchdog", daemon=True).start()
    t0 = time.perf_counter()
    try:
        n = 4096
        x = torch.full((n,), float(tp.rank + 1), dtype=torch.float32, device=device)
        saved, tp.peer = tp.peer, None          # the group's own collectives only
        try:
            tp.all_reduce(x)
            g = tp.all_gather_rows(torch.full((1, 8), float(tp.rank), device=device))
        finally:
            tp.peer = saved
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        want = tp.size * (tp.size + 1) / 2
        ok_ar = bool((x.cpu() == want).all())
        ok_ag = bool((g.cpu() == torch.arange(tp.size, dtype=torch.float32).view(-1, 1)).all())
    finally:
        done.set()
    if not (ok_ar and ok_ag):
        raise GroupSelfTestError(f"TP group self-test: wrong collective result on rank {tp.rank} "
                                 f"(all_reduce ok={ok_ar}, all_gather ok={ok_ag})")
    dt = time.perf_counter() - t0
    log.info("TP group self-test ok (%s, %d ranks) in %.2f s", dist.get_backend(tp.group),
             tp.size, dt)
    return {"backend": dist.get_backend(tp.group), "seconds": round(dt, 3)}


def attach_channel(engine, tp: TPContext, tag: str) -> PlanChannel | None:
    """Leader creates the plan mailbox, followers attach after a barrier."""
    if tp.size == 1:
        return None
    path = mailbox_path(tag)
    ch = None
    if tp.rank == 0:
        ch = PlanChannel(path, 0, tp.size, create=True)
    dist.barrier(group=tp.group)
    if tp.rank:
        ch = PlanChannel(path, tp.rank, tp.size, create=False)
    engine.chan = ch
    return ch


def probe_allreduce(tp: TPContext, device: torch.device, sizes=(16 << 10, 256 << 10, 1 << 20,
                                                                4 << 20), iters: int = 20) -> dict:
    """Time the group's all-reduce paths on decode-sized bf16 messages
    (collective: all ranks call it).  Returns {path: {bytes: us}}; exported
    as rccl_allreduce_seconds{group=path} by the serving process."""
    out: dict[str, dict[int, float]] = {}
    paths = [("rccl", None)]
    if tp.peer is not None:
        paths.append(("peer", tp.peer))
    for name, peer in paths:
        res = {}
        for n in sizes:
            x = torch.zeros(n // 2, dtype=torch.bfloat16, device=device)
            if peer is not None and not peer.supports(x):
                continue

            def call():
                if peer is not None:
                    peer(x)
                else:
                    saved, tp.peer = tp.peer, None
                    try:
                        tp.all_reduce(x)
                    finally:
                        tp.peer = saved
            for _ in range(3):
                call()
            if device.type != "cuda":          # gloo group (CPU tests / plumbing)
                t0 = time.perf_counter()
                for _ in range(iters):
                    call()
                res[n] = round((time.perf_counter() - t0) / iters * 1e6, 1)
                continue
            torch.cuda.synchronize(device)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                call()
            e.record()
            torch.cuda.synchronize(device)
            res[n] = round(s.elapsed_time(e) / iters * 1e3, 1)
        out[name] = res
    return out


def build_tp_engine(ecfg, device, tp: TPContext, tag: str, weights_path: str = "",
                    model_cfg=None):
    from ..engine.engine import LLMEngine
    from ..models import config as mc
    cfg = model_cfg or mc.resolve(ecfg.model)
    weights = None
    if weights_path:
        from ..models.weights import load_llama_weights
        weights = load_llama_weights(weights_path, cfg, device, tp.rank, tp.size)
    dev = torch.device(device)
    comm = {}
    selftest = group_self_test(tp, dev) if tp.size > 1 else {}
    if dev.type == "cuda" and tp.size > 1:
        from .peer_allreduce import setup as setup_peer_ar
        setup_peer_ar(tp, dev)
        comm = probe_allreduce(tp, dev)
        log.info("TP all-reduce us by message size: %s", comm)
    eng = LLMEngine(ecfg, device=device, model_cfg=cfg, tp=tp, weights=weights)
    eng.tp_comm = comm
    eng.tp_selftest = selftest
    attach_channel(eng, tp, tag)
    return eng


def run_tp_worker(a) -> None:
    """Entry from worker/main.py when ``--tp N`` (one call per rank)."""
    from ..devices import rocm_enum
    from ..engine.engine import EngineConfig
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if getattr(a, "cpu", False):
        dev = torch.device("cpu")      # gloo group (tests / plumbing)
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    tp = init_group(dev)
    if tp.size != a.tp:
        raise SystemExit(f"--tp {a.tp} but the launcher started {tp.size} ranks")
    ecfg = EngineConfig(model=a.chat_model, max_num_seqs=a.max_num_seqs,
                        max_model_len=a.max_model_len, kv_fraction=a.kv_fraction)
    if a.max_batched_tokens:
        ecfg.max_batched_tokens = a.max_batched_tokens
    tag = f"{rocm_enum.host_id()}-{os.environ.get('MASTER_PORT', '0')}"
    engine = build_tp_engine(ecfg, dev, tp, tag, a.weights)
    log.info("TP rank %d/%d ready: %d KV blocks, %d graphs", tp.rank, tp.size,
             engine.num_blocks, len(engine.graphs))
    try:
        if tp.rank == 0:
            from ..worker.main import serve_engines
            vis = os.environ.get("HIP_VISIBLE_DEVICES", "")
            gpus = vis.split(",") if vis else [str(i) for i in range(tp.size)]
            device_id = f"{rocm_enum.host_id()}:tp{tp.size}:gpu{gpus[0]}-{gpus[-1]}"
            try:
                serve_engines(a, engine, None, device_id)
            finally:
                engine.release_followers()
        else:
            try:
                engine.run_follower()
            except LeaderLost as e:
                # the group is gone: exit non-zero at once (a collective
                # teardown could wait forever on the dead leader) so the
                # launcher ends the group and the supervisor starts a new one
                log.error("TP rank %d: %s; exiting", tp.rank, e)
                logging.shutdown()
                os._exit(3)
    finally:
        if engine.chan is not None:
            engine.chan.close()
        dist.destroy_process_group()
