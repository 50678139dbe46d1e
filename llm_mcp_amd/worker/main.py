"""GPU worker process: ``python -m llm_mcp_amd.worker.main --gpu 0 ...``.

Owns one MI355X (or, with --tp N, leads a tensor-parallel group launched by
torch.distributed.run): builds the chat engine (and optionally the embedding
engine) on its device, serves the synchronous OpenAI path to the API process
over a Unix socket (engine/ipc.py) and claims async jobs from the core over
gRPC, executing them in-process on the same continuous-batching engine.
Replaces worker/llm_worker/main.py (which forwarded every job to Ollama over
HTTP)."""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal

log = logging.getLogger("lmx.worker")


SHARED_GPU_BATCHED_TOKENS = 8192   # prefill budget of a chat engine sharing its GPU


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", type=int, default=int(os.environ.get("LOCAL_RANK", "0")))
    ap.add_argument("--chat-model", default=os.environ.get("LMX_CHAT_MODEL", "llama-3-8b"))
    ap.add_argument("--embed-model", default=os.environ.get("LMX_EMBED_MODEL", ""))
    ap.add_argument("--socket", default="")
    ap.add_argument("--core", default=os.environ.get("CORE_GRPC_ADDR", "127.0.0.1:9090"))
    ap.add_argument("--no-jobs", action="store_true", help="serve the sync path only")
    ap.add_argument("--max-num-seqs", type=int, default=int(os.environ.get("LMX_MAX_BATCH", "256")))
    ap.add_argument("--max-batched-tokens", type=int, default=None,
                    help="default: LMX_MAX_BATCHED_TOKENS (engine.EngineConfig, shared with bench.py)")
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--kv-fraction", type=float, default=0.6)
    ap.add_argument("--lease-seconds", type=int, default=int(os.environ.get("WORKER_LEASE_SECONDS", "60")))
    ap.add_argument("--weights", default="", help="safetensors dir of real weights (optional)")
    ap.add_argument("--embed-weights", default="",
                    help="safetensors dir of the embedding model (nomic-bert or BERT; optional)")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--cpu", action="store_true",
                    help="run the engines on the CPU (tests / plumbing; device ids stay gpuN)")
    ap.add_argument("--replica", type=int, default=0,
                    help="k-th worker on the same GPU (1-GPU rehearsals of multi-GPU serving): "
                         "device id gpuN.rk")
    return ap


def main(argv=None):
    a = build_parser().parse_args(argv)
    logging.basicConfig(level=os.environ.get("LOG_LEVEL", "INFO"))
    if a.tp > 1:
        from ..parallel.tp_worker import run_tp_worker
        return run_tp_worker(a)
    import torch

    from ..devices import rocm_enum
    from ..engine.engine import EngineConfig, LLMEngine
    from ..models import config as mc

    if a.cpu:
        dev = torch.device("cpu")
    else:
        torch.cuda.set_device(a.gpu)
        dev = torch.device("cuda", a.gpu)
    engine = embed = None
    if a.embed_model:
        from ..engine.embed_engine import EmbeddingEngine
        ecfg_e = mc.resolve(a.embed_model)
        ew = None
        if a.embed_weights:
            from ..models.bert import load_bert_weights
            from ..models.nomic_bert import load_nomic_weights
            loader = load_bert_weights if isinstance(ecfg_e, mc.BertConfig) else load_nomic_weights
            ew = loader(a.embed_weights, ecfg_e, dev)
        embed = EmbeddingEngine(ecfg_e, dev, weights=ew)
    if a.chat_model:
        cfg = mc.resolve(a.chat_model)
        weights = None
        if a.weights:
            from ..models.weights import load_llama_weights
            weights = load_llama_weights(a.weights, cfg, dev)
        ecfg = EngineConfig(model=a.chat_model, max_num_seqs=a.max_num_seqs,
                            max_model_len=a.max_model_len, kv_fraction=a.kv_fraction)
        if a.max_batched_tokens:
            ecfg.max_batched_tokens = a.max_batched_tokens
        elif (a.embed_model or a.replica) and not os.environ.get("LMX_MAX_BATCHED_TOKENS"):
            # the GPU is shared: with an embedding engine in this worker, or with other
            # workers on the same card (--replica), a 24k-token prefill step (~235 ms)
            # holds the other engine's batches behind it.  Config 5 (two chat + embed
            # workers on one GPU, faults on one): 73.2 jobs/s mean over nine runs at 8192,
            # 67.6 over six at 24576, with a wide run-to-run spread (profiles/r5_config5.md).
            # A chat-only worker keeps the bench's budget.
            ecfg.max_batched_tokens = SHARED_GPU_BATCHED_TOKENS
        if a.embed_model:
            ecfg.kv_fraction = min(ecfg.kv_fraction, 0.5)
        engine = LLMEngine(ecfg, device=dev, model_cfg=cfg, weights=weights)
    dev_id = rocm_enum.device_id(a.gpu) + (f".r{a.replica}" if a.replica else "")
    serve_engines(a, engine, embed, dev_id)


def serve_engines(a, engine, embed, device_id: str) -> None:
    """Serve a chat engine and/or an embedding engine: the sync OpenAI path
    over the Unix socket and the async job path via lease claims.  Used by the
    single-GPU worker and by the leader of a TP group."""
    from ..api.registry import LocalModel, ModelRegistry
    from ..devices import rocm_enum
    from ..engine.async_engine import AsyncEngine
    from ..engine.ipc import EngineServer
    from ..models.tokenizer import for_model
    from .agent import WorkerAgent, engine_admission
    from .jobs import JobRunner

    fdev = os.environ.get("LMX_FAULT_DEVICE", "")
    lives = int(os.environ.get("LMX_FAULT_LIVES", "0") or 0)
    life = int(os.environ.get("LMX_WORKER_LIFE", "1") or 1)
    if (fdev and not device_id.endswith(fdev)) or (lives > 0 and life > lives):
        from ..utils.faults import Faults, set_faults
        # LMX_FAULT applies to the targeted device only, and (LMX_FAULT_LIVES)
        # only to the first N lives of its worker (the supervisor numbers them)
        set_faults(Faults(""))
    reg = ModelRegistry()
    aeng = None
    if embed is not None:
        reg.add(LocalModel(a.embed_model, "embed", device_id, embed,
                           for_model(embed.cfg), embed.cfg, embed.max_seq_len, capacity=1024))
    if engine is not None:
        aeng = AsyncEngine(engine)
        reg.add(LocalModel(a.chat_model, "chat", device_id, aeng, for_model(engine.cfg),
                           engine.cfg, engine.max_model_len, capacity=a.max_num_seqs))
    sock = a.socket or f"/tmp/lmx-{rocm_enum.host_id()}-{device_id.rsplit(':', 1)[-1]}.sock"
    info = {"device_id": device_id, "models": {}}
    if engine is not None:
        info["models"][a.chat_model] = {"kind": "chat", "max_model_len": engine.max_model_len,
                                        "capacity": a.max_num_seqs,
                                        "tp": engine.tp.size}
    if embed is not None:
        info["models"][a.embed_model] = {"kind": "embed", "max_model_len": embed.max_seq_len,
                                         "capacity": 1024}
    server = EngineServer(engine, sock, info, embed_engine=embed,
                          fallback_sink=aeng._sink if aeng is not None else None)
    if engine is not None:
        engine.event_sink = server._sink

    async def run():
        loop = asyncio.get_running_loop()
        if aeng is not None:
            aeng.loop = loop
        server.start()
        log.info("%s serving %s on %s", device_id, list(info["models"]), sock)
        stop = asyncio.Event()
        for sig in (signal.SIGINT, signal.SIGTERM):
            loop.add_signal_handler(sig, stop.set)
        agent = None
        if not a.no_jobs:
            from ..rpc.client import CoreClient
            client = CoreClient(a.core)

            def mark_offline(dev_id, reason):
                import json
                import urllib.request
                url = os.environ.get("CORE_HTTP_URL", "http://127.0.0.1:8080").rstrip("/")
                req = urllib.request.Request(url + "/v1/devices/offline", method="POST",
                                             data=json.dumps({"device_id": dev_id,
                                                              "reason": reason}).encode(),
                                             headers={"Content-Type": "application/json"})
                urllib.request.urlopen(req, timeout=5).read()

            runner = JobRunner(reg, device_id,
                               report_benchmark=lambda **kw: client.report_benchmark(**kw))
            agent = WorkerAgent(client, runner, device_id,
                                worker_id=os.environ.get("WORKER_ID", f"worker-{device_id}"),
                                lease_s=a.lease_seconds, capacity=a.max_num_seqs,
                                tags={"engine": True, "models": list(info["models"])},
                                mark_offline=mark_offline,
                                health=engine.healthy if engine is not None else None,
                                admit=engine_admission(engine) if engine is not None else None)
            task = asyncio.create_task(agent.run())
        fatal = {}

        async def watchdog():
            # an engine error (HIP fault) or a hung step is fatal for this GPU
            # process: stop, let the in-flight leases lapse / requeue, exit
            # non-zero -- the serve supervisor starts a fresh worker
            while engine is not None and not stop.is_set():
                await asyncio.sleep(WATCHDOG_S)
                ok, why = engine.healthy()
                if not ok:
                    log.error("%s unhealthy: %s; worker exits for a restart", device_id, why)
                    fatal["why"] = why
                    await asyncio.sleep(WATCHDOG_GRACE_S)   # let in-flight failures report
                    stop.set()

        wd = asyncio.create_task(watchdog())
        await stop.wait()
        wd.cancel()
        if agent is not None:
            agent.stop()
            task.cancel()
        if fatal:
            logging.shutdown()
            os._exit(3)        # no teardown on a broken device (it may hang)
        server.stop()

    asyncio.run(run())


WATCHDOG_S = float(os.environ.get("LMX_WATCHDOG_S", "1.0"))
WATCHDOG_GRACE_S = float(os.environ.get("LMX_WATCHDOG_GRACE_S", "2.0"))


if __name__ == "__main__":
    main()
