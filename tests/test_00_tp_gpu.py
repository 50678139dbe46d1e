"""Tensor-parallel engine group on the GPU kernels (runs first in the GPU
session: the rank processes are spawned before this pytest process touches
the device).

A 1-GPU box cannot host two RCCL ranks, so the two ranks share cuda:0 over a
gloo process group (device tensors staged through the host where gloo needs
it).  Everything else is the production TP path (the all-reduces run on
the peer-memory kernel, parallel/peer_allreduce.py, whose IPC regions the two
processes map on the same device): per-rank shards from the HF
safetensors loader, the leader's plan mailbox, the HIP kernels on each shard,
all-reduces after the O and down projections and the vocab-split LM head."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

PROMPTS = [list(range(10, 50)), list(range(5, 100)), [7] * 33, [3]]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, size, port, ckpt, tag, q, model="tiny-llama", graphs=False, lookahead="0"):
    # sequence parallelism forced on every prefill step of >= 16 tokens (the
    # gloo group takes its host-staged reduce-scatter / all-gather branch)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(size), LOCAL_RANK=str(rank), LMX_SP_MIN_TOKENS="16",
                      LMX_LOOKAHEAD=lookahead)
    import torch.distributed as dist

    from llm_mcp_amd.engine.engine import EngineConfig, SamplingParams
    from llm_mcp_amd.parallel.tp_worker import build_tp_engine, init_group
    torch.cuda.set_device(0)
    tp = init_group("cpu")   # gloo group, GPU tensors
    ecfg = EngineConfig(model=model, max_num_seqs=8, max_batched_tokens=64,
                        max_model_len=512, use_graphs=graphs, kv_cache_gb=0.05)
    eng = build_tp_engine(ecfg, torch.device("cuda", 0), tp, tag, weights_path=ckpt)
    try:
        if rank == 0:
            out = eng.generate(PROMPTS, SamplingParams(temperature=0, max_tokens=6,
                                                       ignore_eos=True))
            eng.release_followers()
            q.put(("leader", out))
            q.put(("comm", eng.tp_comm))
            q.put(("graph_steps", eng.stats["graph_steps"]))
        else:
            q.put((f"follower{rank}", eng.run_follower()))
    finally:
        eng.chan.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("size,model", [(2, "tiny-llama"), (4, "tiny-llama-tp8"),
                                        (8, "tiny-llama-tp8")])
def test_tp_group_on_gpu_kernels(tmp_path, size, model):
    """TP=2, and TP=4 / TP=8 of the 70B-shaped tiny model (4 q / 2 kv and 2 q / 1 kv
    heads per rank): the TP=8 leader/follower group and its world-8 peer
    all-reduce, eight processes on the one GPU."""
    from llm_mcp_amd.models import config as mc
    from llm_mcp_amd.models.llama import LlamaModel
    from llm_mcp_amd.models.weights import save_hf_llama
    from tests.dense_ref import assert_greedy_consistent
    cfg = mc.resolve(model)
    full = LlamaModel(cfg, "cpu", seed=11)          # CPU only in this process
    save_hf_llama(full.w, cfg, str(tmp_path))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tag = f"gputest-{os.getpid()}-{_free_port()}"
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, size, port, str(tmp_path), tag, q, model),
                         daemon=True) for r in range(size)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=400) for _ in range(len(procs) + 2))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    assert all(res[f"follower{r}"] > 0 for r in range(1, size))
    # the all-reduces ran on the peer-memory kernel (IPC regions on the one GPU)
    assert res["comm"].get("peer"), res["comm"]
    for prompt, out in zip(PROMPTS, res["leader"]):
        assert len(out) == 6
        assert_greedy_consistent(full, prompt, out)


def _run_group(tmp_path, size, model, graphs, lookahead):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    tag = f"gputest-{os.getpid()}-{_free_port()}"
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, size, port, str(tmp_path), tag, q, model,
                                             graphs, lookahead), daemon=True)
             for r in range(size)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=400) for _ in range(len(procs) + 2))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.parametrize("size,model,lookahead", [(2, "tiny-llama", "0"), (2, "tiny-llama", "1"),
                                                  (4, "tiny-llama-tp8", "1")])
def test_tp_group_captured_decode_graphs(tmp_path, size, model, lookahead):
    """The TP decode step captured into hipGraphs with the peer-memory all-reduce /
    logits all-gather kernels inside (a gloo group on one GPU: every decode
    collective is a peer kernel, so the engine captures): graph steps run, with
    and without TP lookahead (every rank samples from the all-gathered logits),
    and the greedy tokens equal the eager TP path's."""
    from llm_mcp_amd.models import config as mc
    from llm_mcp_amd.models.llama import LlamaModel
    from llm_mcp_amd.models.weights import save_hf_llama
    cfg = mc.resolve(model)
    full = LlamaModel(cfg, "cpu", seed=11)
    save_hf_llama(full.w, cfg, str(tmp_path))
    eager = _run_group(tmp_path, size, model, False, "0")
    graph = _run_group(tmp_path, size, model, True, lookahead)
    assert eager["graph_steps"] == 0
    assert graph["graph_steps"] > 0, graph
    assert graph["comm"].get("peer"), graph["comm"]
    assert all(graph[f"follower{r}"] > 0 for r in range(1, size))
    assert graph["leader"] == eager["leader"]
